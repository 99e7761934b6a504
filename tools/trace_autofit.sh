cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05/n_aftrace; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 bench.py --config af --series 65536 --steps 1 --warmup 0 --cpu-seconds 0 > $O/bench.json 2> $O/bench.err

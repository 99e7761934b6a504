# Kernel trace of one autoFit step (the bench's af config) for the time breakdown per kernel (run ON the GPU box
# from the repo root): TAG names the output directory, SER the series (default 1M, the bench's line)
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r06/${TAG:-ze_aftrace}; mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 bench.py --config af --series ${SER:-1048576} --steps 1 --warmup 0 --cpu-seconds 0 > $O/bench.json 2> $O/bench.err

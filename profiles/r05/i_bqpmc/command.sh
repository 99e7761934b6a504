cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05/i_bqpmc; mkdir -p $O
export PROBE_WHAT=bobyqa
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 tools/bobyqa_probe.py 1024 > $O/trace.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_FLAT SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_WAIT_INST_ANY -d $O/p1 -o run --output-format csv -- python3 tools/bobyqa_probe.py 1024 > $O/p1.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_FLAT SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_ANY SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY -d $O/p2 -o run --output-format csv -- python3 tools/bobyqa_probe.py 1024 > $O/p2.log 2>&1

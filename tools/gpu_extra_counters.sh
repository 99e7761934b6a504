cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
timeout -k 10 60 rocprofv3 -L > gpurun_out/counters_list.txt 2>&1
export SPARKTS_ARIMA_LIB=spark-timeseries_amd/libsparkts_arima_dev_base.so
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM -d gpurun_out/pmc_a -o run --output-format csv -- python3 tools/variant_run.py --reps 1 > /dev/null 2> gpurun_out/pmc_a.err &&
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 -d gpurun_out/pmc_b -o run --output-format csv -- python3 tools/variant_run.py --reps 1 > /dev/null 2> gpurun_out/pmc_b.err

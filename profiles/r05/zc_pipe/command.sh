bash tools/trace_c2_pipe.sh; python tools/pipe_overlap.py <kernel_trace.csv> --skip-first 40 > pipe_overlap.txt   # shipped build

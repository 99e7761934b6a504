TAG=d_bobyqa2 TESTS=1 SMOKE=1 BENCH="--config af" BENCH_TIMEOUT=500 bash tools/gpu_session.sh   # tests + smoke green; the af bench (1M series) was killed silent after 180 s: see e_probe

TAG=a_prune TESTS=1 SMOKE=1 BENCH="--steps 20 --warmup 3" BENCH2="--config c1 --steps 20 --warmup 3" BENCH_TIMEOUT=500 bash tools/gpu_session.sh

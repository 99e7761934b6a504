pytest tests/test_gpu_sharded.py -k autofit   # bench --config af on 2 ranks sharing GPU 0, per-rank oracle parity

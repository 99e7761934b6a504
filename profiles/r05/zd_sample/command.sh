pytest tests/test_gpu_parity.py -k "python_mirror_api or sampler"

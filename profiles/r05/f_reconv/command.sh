pytest tests/test_gpu_bobyqa.py tests/test_gpu_autofit.py; python -u tools/bobyqa_probe.py 1024 16384 65536   # BOBYQB evaluations at one reconvergence point

pytest tests/test_gpu_autofit.py -k long; bash tools/trace_autofit.sh (OUT z_aftrace)   # shipped build

pytest test_gpu_autofit/bobyqa/jni_harness; bobyqa_probe.py 1024 65536   # autoFit with the retries asynchronous to the walk (reverted: 15.1 s vs 9.3 s at 65 536)

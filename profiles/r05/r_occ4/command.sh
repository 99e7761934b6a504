wave layout at 4 waves/SIMD (128 VGPRs): bobyqa_probe.py 1024 65536

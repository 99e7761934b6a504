wave layout at 2 waves/SIMD (256 VGPRs): bobyqa_probe.py 1024 65536

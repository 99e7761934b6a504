wave layout with the parallel-in-time objective over the row in LDS (reverted): bobyqa_probe.py 1024 16384 65536

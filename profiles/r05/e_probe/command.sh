python -u tools/bobyqa_probe.py 1024 4096 16384 65536 > probe.jsonl

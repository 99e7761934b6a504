pytest test_gpu_bobyqa+autofit; bobyqa_probe.py 1024 65536 (wave layout, 512 VGPRs) and SPARKTS_OPTIONS=bobyqa_wave=0 (lane layout)

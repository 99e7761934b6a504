pytest test_gpu_bobyqa+autofit; bobyqa_probe.py 1024 4096 65536   # wave layout with the O(npt n) loops split over lanes

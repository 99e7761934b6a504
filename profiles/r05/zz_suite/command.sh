TAG=zz_suite TESTS=1 SMOKE=1 bash tools/gpu_session.sh   # the final tree, shipped library 731448ab

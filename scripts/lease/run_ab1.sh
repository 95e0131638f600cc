bash scripts/gpu_tests.sh -x && VARIANTS=hibranch bash scripts/gpu_ab.sh --configs 2,3 --qs 11 --pairs 1 --labs 0,1 --modes global --rounds 5

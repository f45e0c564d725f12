#!/bin/bash
set -o pipefail
O=gpurun_out/r02s40
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_exhaustive.py tests/test_gpu_parity.py tests/test_gpu_config_fuzz.py tests/test_gpu_velocity.py tests/test_gpu_vec.py tests/test_gpu_env.py tests/test_gpu_state.py > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log
[ $rc -eq 0 ] || exit 1
bash tools/ab_multi.sh cfg2 3 new ab/prev.so && bash tools/ab_multi.sh cfg5 1 new ab/prev.so

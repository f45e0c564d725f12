#!/bin/bash
set -o pipefail
O=gpurun_out/r02s36
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_exhaustive.py tests/test_gpu_parity.py tests/test_gpu_config_fuzz.py > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python tools/stamps.py cfg5 cfg2 > $O/stamps.log 2>&1
grep "channel loop\|phases:" $O/stamps.log
bash tools/ab_multi.sh cfg5 2 new ab/prev.so && bash tools/ab_multi.sh cfg2 2 new ab/prev.so && bash tools/ab_multi.sh cfg4 1 new ab/prev.so

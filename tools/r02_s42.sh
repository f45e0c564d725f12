#!/bin/bash
set -o pipefail
O=gpurun_out/r02s42
mkdir -p $O
timeout -k 10 1000 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests -m gpu > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log
[ $rc -eq 0 ] || exit 1
bash tools/ab_multi.sh cfg5 2 new ab/prev.so && bash tools/ab_multi.sh cfg2 2 new ab/prev.so && bash tools/ab_multi.sh cfg4 1 new ab/prev.so && bash tools/ab_multi.sh cfg3 1 new ab/prev.so

#!/bin/bash
# A/B: the traffic reset's w1/id slot stores by the group's other lanes (new) vs lane 0 (ab/old.so),
# after the traffic parity tests on the new build.
O=gpurun_out/r02s5split
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_traffic_groups.py tests/test_gpu_car_slots.py tests/test_gpu_exhaustive.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
tail -2 $O/tests.log
grep -q " passed" $O/tests.log && ! grep -q "failed\|error" $O/tests.log || exit 1
timeout -k 10 600 bash tools/ab_multi.sh cfg3 4 ab/old.so new | tee $O/ab.txt

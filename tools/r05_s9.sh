#!/bin/bash
# round 5 session 9: 192-env map-queue workgroups (three env waves + helper) -- parity and A/B
set -o pipefail
O=gpurun_out/r05s9; mkdir -p $O
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_exhaustive.py -k "wg192 or cfg5_all or cfg2_all" > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; grep -E "FAILED" $O/pytest.log | head; [ $rc -le 1 ] || exit 1
AB_STEPS=200 timeout -k 10 900 bash tools/ab_multi.sh cfg5 3 new new:--envs-per-block=192 > $O/ab.log 2>&1 || { cat $O/ab.log; exit 1; }
grep -v amdgpu.ids $O/ab.log
for n in 131072 262144; do
  AB_STEPS=400 timeout -k 10 300 bash tools/ab_multi.sh cfg5 2 new:--envs=$n new:--envs=$n:--envs-per-block=192 > $O/ab_$n.log 2>&1 || { cat $O/ab_$n.log; exit 1; }
  grep -v amdgpu.ids $O/ab_$n.log
done

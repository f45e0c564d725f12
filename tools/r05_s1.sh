#!/bin/bash
# round 5 session 1: dual-graph removal test (ab/dual.so) + register-resident exits (new) -- parity, genbench,
# interleaved A/B vs r04
set -o pipefail
mkdir -p gpurun_out/r05s1
O=gpurun_out/r05s1
timeout -k 10 400 python -u -m pytest -v -s --timeout 300 --timeout-method thread tests/test_gpu_map_generator.py tests/test_gpu_exhaustive.py tests/test_gpu_parity.py > $O/pytest.log 2>&1
rc=$?; tail -5 $O/pytest.log; grep -E "FAILED|maps differ" $O/pytest.log | head; [ $rc -le 1 ] || exit 1
for L in ab/r04_stamps.so ab/dual_stamps.so pgtg_amd/libpgtg_hip_stamps.so; do
  PGTG_STAMPS_LIB=$PWD/$L timeout -k 10 120 python tools/genbench.py 5 1024 8 >> $O/genbench.log 2>&1 || exit 1
  PGTG_STAMPS_LIB=$PWD/$L timeout -k 10 120 python tools/genbench.py 3 1024 8 >> $O/genbench.log 2>&1 || exit 1
done
cat $O/genbench.log
AB_STEPS=200 timeout -k 10 600 bash tools/ab_multi.sh cfg5 3 ab/r04.so ab/dual.so new > $O/ab_cfg5.log 2>&1 || { cat $O/ab_cfg5.log; exit 1; }
cat $O/ab_cfg5.log
AB_STEPS=400 timeout -k 10 300 bash tools/ab_multi.sh cfg2 2 ab/r04.so ab/dual.so new > $O/ab_cfg2.log 2>&1 || { cat $O/ab_cfg2.log; exit 1; }
cat $O/ab_cfg2.log

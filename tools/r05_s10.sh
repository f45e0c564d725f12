#!/bin/bash
# round 5 session 10: batched removal draws -- map parity, genbench vs the previous build, A/B
set -o pipefail
O=gpurun_out/r05s10; mkdir -p $O
timeout -k 10 400 python -u -m pytest -v -s --timeout 300 --timeout-method thread tests/test_gpu_map_generator.py > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; grep -E "FAILED|maps differ" $O/pytest.log | head -3; [ $rc -le 1 ] || exit 1
for L in ab/dual_stamps.so pgtg_amd/libpgtg_hip_stamps.so; do
  PGTG_STAMPS_LIB=$PWD/$L timeout -k 10 120 python tools/genbench.py 5 1024 8 2>&1 | grep -v amdgpu.ids || exit 1
done
AB_STEPS=200 timeout -k 10 900 bash tools/ab_multi.sh cfg5 3 ab/pre_batch.so new ab/pre_batch.so:--envs-per-block=192 new:--envs-per-block=192 > $O/ab.log 2>&1 || { cat $O/ab.log; exit 1; }
grep -v amdgpu.ids $O/ab.log

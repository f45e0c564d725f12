#!/bin/bash
# round 5 session 2: in-situ chains (stamps) of k_envq r04 vs new, and the refill ablation on the new tree
set -o pipefail
O=gpurun_out/r05s2; mkdir -p $O
for L in ab/r04_stamps.so pgtg_amd/libpgtg_hip_stamps.so; do
  echo "== $L" >> $O/stamps.log
  PGTG_STAMPS_LIB=$PWD/$L timeout -k 10 120 python tools/stamps.py cfg5big cfg2 >> $O/stamps.log 2>&1 || { cat $O/stamps.log; exit 1; }
done
grep -v amdgpu.ids $O/stamps.log
timeout -k 10 900 bash tools/ablate.sh r05s2/abl cfg5 2>&1 | grep -v amdgpu.ids

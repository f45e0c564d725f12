#!/bin/bash
# round 5 session 8: what the helper wave costs the launch -- spin (issue only) vs refills vs refills without stores
set -o pipefail
O=gpurun_out/r05s8; mkdir -p $O
T=pgtg_amd/libpgtg_hip_tuning.so
AB_STEPS=200 timeout -k 10 900 bash tools/ab_multi.sh cfg5 2 $T:PGTG_ABL=0 $T:PGTG_ABL=1 $T:PGTG_ABL=16 $T:PGTG_ABL=8:PGTG_SPIN=2000 $T:PGTG_ABL=8:PGTG_SPIN=4000 $T:PGTG_ABL=8:PGTG_SPIN=8000 > $O/ab.log 2>&1 || { cat $O/ab.log; exit 1; }
grep -v amdgpu.ids $O/ab.log

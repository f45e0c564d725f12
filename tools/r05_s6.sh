#!/bin/bash
# round 5 session 6: stamps of the traffic workloads (where k_env<true>'s time goes)
set -o pipefail
O=gpurun_out/r05s6; mkdir -p $O
PGTG_STAMP_STEPS=60 timeout -k 10 200 python tools/stamps.py cfg3 train > $O/stamps.log 2>&1 || { tail -20 $O/stamps.log; exit 1; }
grep -v amdgpu.ids $O/stamps.log

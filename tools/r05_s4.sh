#!/bin/bash
# round 5 session 4: the in-place reset kernels (k_env) r04 vs new: configs[3], configs[2], caller workload
set -o pipefail
O=gpurun_out/r05s4; mkdir -p $O
AB_STEPS=200 timeout -k 10 400 bash tools/ab_multi.sh cfg4 3 ab/r04.so new > $O/ab_cfg4.log 2>&1 || { cat $O/ab_cfg4.log; exit 1; }
grep -v amdgpu.ids $O/ab_cfg4.log
AB_STEPS=100 AB_WARMUP=50 timeout -k 10 400 bash tools/ab_multi.sh train 2 ab/r04.so new > $O/ab_train.log 2>&1 || { cat $O/ab_train.log; exit 1; }
grep -v amdgpu.ids $O/ab_train.log
AB_STEPS=100 AB_WARMUP=100 timeout -k 10 400 bash tools/ab_multi.sh cfg3 2 ab/r04.so new > $O/ab_cfg3.log 2>&1 || { cat $O/ab_cfg3.log; exit 1; }
grep -v amdgpu.ids $O/ab_cfg3.log

#!/bin/bash
# Interleaved bench lines of several builds on one box.  Usage: bash tools/ab_multi.sh <workload> <reps> <lib.so|new>...
W=$1; R=$2; shift 2
mkdir -p gpurun_out
for rep in $(seq $R); do
  for L in "$@"; do
    if [ $L = new ]; then unset PGTG_LIB; else export PGTG_LIB=$PWD/$L; fi
    timeout -k 10 120 python bench.py --workload $W --steps ${AB_STEPS:-100} --warmup ${AB_WARMUP:-20} --no-cpu-baseline > gpurun_out/abm.json || exit 1
    python -c "import json; d=json.load(open('gpurun_out/abm.json')); r=d['roofline']; print('$W $L', f\"{d['value']/1e6:.2f}M\", f\"kern {r['avg_kernel_us']:.1f}us\")"
  done
done

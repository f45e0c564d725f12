#!/bin/bash
# A/B: first-round start offsets (stagger_start) by batch size, through the PGTG_TUNING build's
# PGTG_STAGGER knob.  Usage: bash tools/stagger_ab.sh <reps> <envs>...
R=$1; shift
export PGTG_LIB=$PWD/pgtg_amd/libpgtg_hip_tuning.so
for rep in $(seq $R); do
  for N in "$@"; do
    for ST in 0 1; do
      PGTG_STAGGER=$ST timeout -k 10 120 python bench.py --envs $N --steps 300 --warmup 20 --no-cpu-baseline > gpurun_out/stg.json || exit 1
      python -c "import json; d=json.load(open('gpurun_out/stg.json')); r=d['roofline']; print('envs $N stagger $ST', f\"{d['value']/1e6:.1f}M\", f\"kern {r['avg_kernel_us']:.1f}us\")"
    done
  done
done

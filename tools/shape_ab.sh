#!/bin/bash
# A/B: bench lines of one batch size under several step-kernel shapes.  Usage: bash tools/shape_ab.sh <envs> <reps> <envs-per-block>...
N=$1; R=$2; shift 2
for rep in $(seq $R); do
  for E in "$@"; do
    timeout -k 10 120 python bench.py --envs $N --steps 300 --warmup 20 --no-cpu-baseline --envs-per-block $E > gpurun_out/shp.json || exit 1
    python -c "import json; d=json.load(open('gpurun_out/shp.json')); r=d['roofline']; print('envs $N per-block $E', f\"{d['value']/1e6:.1f}M\", f\"kern {r['avg_kernel_us']:.1f}us\", r['kernel'])"
  done
done

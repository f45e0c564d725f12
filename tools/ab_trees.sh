#!/bin/bash
# Interleaved bench lines of whole source trees (each with its own built library) on one box.
# Usage: bash tools/ab_trees.sh <workload> <reps> <steps> <tree dir>...   ("." = this tree)
W=$1; R=$2; S=$3; shift 3
ROOT=$PWD
mkdir -p gpurun_out
for rep in $(seq $R); do
  for T in "$@"; do
    (cd $T && timeout -k 10 180 python bench.py --workload $W --steps $S --warmup 20 --no-cpu-baseline > $ROOT/gpurun_out/abt.json) || exit 1
    python -c "import json; d=json.load(open('gpurun_out/abt.json')); r=d['roofline']; print('$W $T', f\"{d['value']/1e6:.2f}M\", f\"kern {r['avg_kernel_us']:.1f}us\")"
  done
done

#!/bin/bash
# Interleaved bench lines of the tuning build under different values of one knob.
# Usage: bash tools/ab_env.sh <workload> <reps> <KNOB> <value>...
W=$1; R=$2; K=$3; shift 3
mkdir -p gpurun_out
export PGTG_LIB=$PWD/pgtg_amd/libpgtg_hip_tuning.so
for rep in $(seq $R); do
  for V in "$@"; do
    export $K=$V
    timeout -k 10 120 python bench.py --workload $W --steps 100 --warmup 20 --no-cpu-baseline > gpurun_out/abe.json || exit 1
    python -c "import json; d=json.load(open('gpurun_out/abe.json')); r=d['roofline']; print('$W $K=$V', f\"{d['value']/1e6:.2f}M\", f\"kern {r['avg_kernel_us']:.1f}us\", flush=True)"
  done
done

#!/bin/bash
# A/B of the first-round start offsets (PGTG_STAGGER, 100 MHz ticks) on the tuning build, interleaved.
# Usage: bash tools/r02_stagger.sh <workload> <envs|0> <reps> <ticks>...
W=$1; N=$2; R=$3; shift 3
mkdir -p gpurun_out
export PGTG_LIB=$PWD/pgtg_amd/libpgtg_hip_tuning.so
for rep in $(seq $R); do
  for T in "$@"; do
    export PGTG_STAGGER=$T
    timeout -k 10 120 python bench.py --workload $W --envs $N --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/stg.json || exit 1
    python -c "import json; d=json.load(open('gpurun_out/stg.json')); r=d['roofline']; print('$W n=$N stagger=$T', f\"{d['value']/1e6:.1f}M\", f\"kern {r['avg_kernel_us']:.1f}us\", f\"frac {r['frac']:.3f}\", flush=True)"
  done
done

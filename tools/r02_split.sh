#!/bin/bash
# A/B of the split observation writes (PGTG_SPLIT) x stagger on the tuning build, interleaved.
# Usage: bash tools/r02_split.sh <workload> <envs|0> <reps> "<split>:<stagger>"...
W=$1; N=$2; R=$3; shift 3
mkdir -p gpurun_out
export PGTG_LIB=$PWD/pgtg_amd/libpgtg_hip_tuning.so
for rep in $(seq $R); do
  for V in "$@"; do
    export PGTG_SPLIT=${V%%:*} PGTG_STAGGER=${V##*:}
    timeout -k 10 120 python bench.py --workload $W --envs $N --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/spl.json || exit 1
    python -c "import json; d=json.load(open('gpurun_out/spl.json')); r=d['roofline']; print('$W n=$N split:stagger=$V', f\"{d['value']/1e6:.1f}M\", f\"kern {r['avg_kernel_us']:.1f}us\", f\"frac {r['frac']:.3f}\", flush=True)"
  done
done

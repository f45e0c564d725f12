#!/bin/bash
# Bench one workload under tuning-knob settings.  Usage: bash tools/knobs.sh <workload> "K=V K=V" "K=V" ...
W=$1; shift
mkdir -p gpurun_out
for S in "$@"; do
  env $S timeout -k 10 120 python bench.py --workload $W --steps 100 --warmup 20 --no-cpu-baseline > gpurun_out/knob.json || exit 1
  python -c "import json; d=json.load(open('gpurun_out/knob.json')); r=d['roofline']; print('$W [$S]', f\"{d['value']/1e6:.1f}M\", f\"kern {r['avg_kernel_us']:.1f}us\", 'epb', r['envs_per_workgroup'], 'wg/CU', r.get('workgroups_per_cu'))"
done

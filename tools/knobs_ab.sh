#!/bin/bash
# Interleaved A/B of knob settings on one workload (3 rounds).  Usage: bash tools/knobs_ab.sh <workload> "K=V" "K=V" ...
W=$1; shift
for r in 1 2 3; do
  for S in "$@"; do
    env $S timeout -k 10 120 python bench.py --workload $W --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/knob.json || exit 1
    python -c "import json; d=json.load(open('gpurun_out/knob.json')); r=d['roofline']; print('$W [$S]', f\"{d['value']/1e6:.1f}M\", f\"kern {r['avg_kernel_us']:.1f}us\")"
  done
done

#!/bin/bash
# Quick bench of the given workloads (default: all four), one line each.  Usage: bash tools/bench_quick.sh [tag] [workloads...]
set -e
TAG=${1:-dev}; shift || true
WLS=${@:-cfg2 cfg4 cfg5 cfg3}
mkdir -p gpurun_out
for W in $WLS; do
  timeout -k 10 120 python bench.py --workload $W --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/q_${TAG}_$W.json
  python -c "import json; d=json.load(open('gpurun_out/q_${TAG}_$W.json')); r=d['roofline']; print('$W', f\"{d['value']/1e6:.1f}M env-steps/s\", f\"kernel {r['avg_kernel_us']:.1f}us\", f\"frac {r['frac']:.3f}\", 'wg/CU', r.get('workgroups_per_cu'), 'lds', r['lds_bytes'])"
done

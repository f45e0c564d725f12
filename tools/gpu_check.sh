#!/bin/bash
# One GPU session: parity tests, smoke, benches, rocprofv3 kernel stats.  Usage: bash tools/gpu_check.sh [tag]
set -e
TAG=${1:-dev}
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q 2>&1 | tail -15
timeout -k 10 300 python -c "import __graft_entry__ as g; g.build(); g.smoke()"
for W in cfg2 cfg4 cfg5 cfg3; do
  timeout -k 10 300 python bench.py --workload $W --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/bench_${TAG}_$W.json
  python -c "import json; d=json.load(open('gpurun_out/bench_${TAG}_$W.json')); r=d['roofline']; print('$W', f\"{d['value']/1e6:.1f}M env-steps/s\", f\"kernel {r['avg_kernel_us']:.1f}us\", f\"{r['achieved']:.1f} GB/s frac {r['frac']:.4f}\")"
done
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG} -o run --output-format csv -- python bench.py --steps 200 --warmup 20 --no-cpu-baseline > /dev/null
cat gpurun_out/prof_${TAG}/run_kernel_stats.csv | cut -c1-200 | head -4

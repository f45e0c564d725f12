#!/bin/bash
# Quick per-workload bench lines: value, kernel us, ms/step, envs per workgroup.
set -e
for W in ${@:-cfg2 cfg4 cfg5 cfg3}; do
  timeout -k 10 120 python bench.py --workload $W --steps 200 --warmup 20 --no-cpu-baseline $BENCH_ARGS > gpurun_out/ba_$W.json
  python -c "import json; d=json.load(open('gpurun_out/ba_$W.json')); r=d['roofline']; print('$W', round(d['value']/1e6,1), 'M/s kernel', round(r['avg_kernel_us'],1), 'us step', round(d['ms_per_step']*1000,1), 'us E', r['envs_per_workgroup'], 'frac', round(r['frac'],4))"
done

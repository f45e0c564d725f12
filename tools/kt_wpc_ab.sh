#!/bin/bash
# k_traffic workgroups per CU (bench.py --kt-wpc): interleaved bench lines of the caller workload and
# configs[2].  Usage: bash tools/kt_wpc_ab.sh [wpc values...]
for W in train cfg3; do for rep in 1 2; do for K in ${@:-1 2}; do
  timeout -k 10 120 python bench.py --workload $W --steps 200 --warmup 20 --no-cpu-baseline --kt-wpc $K > gpurun_out/ktw.json || exit 1
  python -c "import json; d=json.load(open('gpurun_out/ktw.json')); print('$W kt_wpc=$K', round(d['value']/1e6,2), 'M', round(d['roofline']['avg_kernel_us'],1), 'us')"
done; done; done

#!/bin/bash
# LDS/occupancy experiment: observation sub-batch size for the large no-traffic workloads.
set -e
for SUB in 0 128 64; do
  for W in cfg4 cfg5; do
    if [ $SUB = 0 ]; then unset PGTG_OBS_SUB; else export PGTG_OBS_SUB=$SUB; fi
    timeout -k 10 120 python bench.py --workload $W --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/ss_${W}_$SUB.json
    python -c "import json; d=json.load(open('gpurun_out/ss_${W}_$SUB.json')); r=d['roofline']; print('$W sub=$SUB', round(d['value']/1e6,1), round(r['avg_kernel_us'],1), r['lds_bytes'])"
  done
done

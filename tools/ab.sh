#!/bin/bash
# A/B bench of the in-tree library against another build.  Usage: bash tools/ab.sh <other.so> <workloads...>
O=$1; shift
for W in "$@"; do
  for L in new old new old; do
    if [ $L = new ]; then unset PGTG_LIB; else export PGTG_LIB=$PWD/$O; fi
    timeout -k 10 120 python bench.py --workload $W --steps 100 --warmup 20 --no-cpu-baseline > gpurun_out/ab.json || exit 1
    python -c "import json; d=json.load(open('gpurun_out/ab.json')); r=d['roofline']; print('$W $L', f\"{d['value']/1e6:.1f}M\", f\"kern {r['avg_kernel_us']:.1f}us\", 'wg/CU', r.get('workgroups_per_cu'))"
  done
done

#!/bin/bash
# A/B: k_traffic duration by launch shape (rocprofv3 kernel stats).  Usage: bash tools/kt_shapes.sh "<bench args>"...
export TMPDIR=/tmp
i=0
mkdir -p gpurun_out/kts
for A in "$@"; do
  i=$((i+1))
  D=gpurun_out/kts/$i
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $D -o run --output-format csv -- python bench.py --workload cfg3 --steps 40 --warmup 10 --no-cpu-baseline $A > $D.json 2>$D.err || exit 1
  python -c "
import csv,glob,json
f=glob.glob('$D/**/run_kernel_stats.csv', recursive=True)[0]
v=json.loads(open('$D.json').read().strip().splitlines()[-1])['value']/1e6
out=[]
for r in csv.DictReader(open(f)):
    if 'k_env' in r['Name'] or 'k_traffic' in r['Name']: out.append(r['Name'][6:16] + ' %.1f (min %.1f)' % (float(r['AverageNs'])/1e3, float(r['MinNs'])/1e3))
print('$A', round(v,2), 'M', out)
"
done

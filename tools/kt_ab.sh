#!/bin/bash
# Per-kernel rocprofv3 averages of one workload under two builds (in-tree library vs <lib>), for A/B
# runs whose summed time hides which kernel moved.  Usage: bash tools/kt_ab.sh <tag> <workload> <lib.so>
O=gpurun_out/$1; W=$2; L=$3; mkdir -p $O
export TMPDIR=/tmp
for name in new base; do
  if [ $name = new ]; then unset PGTG_LIB; else export PGTG_LIB=$PWD/$L; fi
  timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/kt_$name -o run --output-format csv -- python bench.py --workload $W --steps 400 --warmup 200 --no-cpu-baseline > $O/kt_$name.json 2> $O/kt_$name.err || { tail -5 $O/kt_$name.err; exit 1; }
  f=$(find $O/kt_$name -name "*kernel_stats.csv" | head -1)
  echo "== $name"; python -c "
import csv
for r in csv.DictReader(open('$f')):
    if 'k_' in r['Name']: print(f\"{r['Name'][:40]:40s} calls {r['Calls']:>6s} avg {float(r['AverageNs'])/1e3:8.1f} us\")"
done

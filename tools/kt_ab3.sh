#!/bin/bash
# Per-kernel rocprofv3 averages of one workload under several builds (in-tree library first), for
# A/B runs whose summed time hides which kernel moved.  Usage: bash tools/kt_ab3.sh <tag> <workload> <lib.so>...
O=gpurun_out/$1; W=$2; shift 2; mkdir -p $O
export TMPDIR=/tmp
for rep in 1 2; do
for L in new "$@"; do
  name=$(basename $L .so)_$rep
  if [ $L = new ]; then unset PGTG_LIB; else export PGTG_LIB=$PWD/$L; fi
  timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/kt_$name -o run --output-format csv -- python bench.py --workload $W --steps 400 --warmup 200 --no-cpu-baseline > $O/kt_$name.json 2> $O/kt_$name.err || { tail -5 $O/kt_$name.err; exit 1; }
  f=$(find $O/kt_$name -name "*kernel_stats.csv" | head -1)
  python -c "
import csv
print('$name', '  '.join(f\"{r['Name'][:18]} {float(r['AverageNs'])/1e3:.1f}\" for r in csv.DictReader(open('$f')) if 'k_env' in r['Name'] or 'k_traffic' in r['Name']))"
done
done

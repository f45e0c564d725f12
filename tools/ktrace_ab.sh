#!/bin/bash
# Per-kernel averages (rocprofv3 kernel trace) of one workload for the in-tree library and another
# build.  Usage: bash tools/ktrace_ab.sh <other.so> <workload>
set -e
export TMPDIR=/tmp
O=$1; W=$2
D=gpurun_out/ktab
mkdir -p $D
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/new -o run --output-format csv -- python bench.py --workload $W --steps 200 --warmup 20 --no-cpu-baseline > /dev/null
PGTG_LIB=$PWD/$O timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/old -o run --output-format csv -- python bench.py --workload $W --steps 200 --warmup 20 --no-cpu-baseline > /dev/null
python tools/kstats.py $(find $D/new -name "*kernel_stats.csv") $(find $D/old -name "*kernel_stats.csv")

#!/bin/bash
# Instruction/scalar cache counters of one workload's step kernel.  Usage: bash tools/icache.sh <tag> <workload> [kernel]
TAG=$1; W=$2; K=${3:-k_env}
export TMPDIR=/tmp
D=gpurun_out/ic_$TAG/$W
mkdir -p $D
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_IFETCH SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_DCACHE_HITS SQC_DCACHE_MISSES"
timeout -s KILL 90 rocprofv3 --pmc $P1 -d $D/p1 -o run --output-format csv -- python bench.py --workload $W --steps 20 --warmup 5 --no-cpu-baseline > /dev/null || exit 1
python tools/sq.py $K $D/p1 | tail -1

#!/bin/bash
# A/B of builds on one box: interleaved bench lines and the two SQ counter passes of the step kernel.
# Usage: bash tools/ab_sq.sh <tag> <workload> <kernel substring> <lib.so|new>...
set -o pipefail
TAG=$1; W=$2; K=$3; shift 3
export TMPDIR=/tmp
D=gpurun_out/absq_$TAG
mkdir -p $D
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU"
P2="SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS"
for rep in 1 2; do
  for L in "$@"; do
    if [ $L = new ]; then unset PGTG_LIB; else export PGTG_LIB=$PWD/$L; fi
    timeout -k 10 120 python bench.py --workload $W --steps 100 --warmup 20 --no-cpu-baseline > $D/b.json || exit 1
    python -c "import json; d=json.load(open('$D/b.json')); r=d['roofline']; print('$W $L', f\"{d['value']/1e6:.2f}M\", f\"kern {r['avg_kernel_us']:.1f}us\")"
  done
done
for L in "$@"; do
  if [ $L = new ]; then unset PGTG_LIB; else export PGTG_LIB=$PWD/$L; fi
  N=$(basename $L .so)
  i=0
  for P in "$P1" "$P2"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $P -d $D/$N/p$i -o run --output-format csv -- python bench.py --workload $W --steps 20 --warmup 5 --no-cpu-baseline > /dev/null || exit 1
  done
  echo "== $L"; python tools/sq.py $K $D/$N/p1 $D/$N/p2 | tail -2
done

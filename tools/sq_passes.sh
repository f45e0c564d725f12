#!/bin/bash
# SQ counter passes (issue/stall breakdown) of one workload's step kernel.  Usage: bash tools/sq_passes.sh <tag> <workload> [kernel substring]
set -e
TAG=$1; W=$2
export TMPDIR=/tmp
D=gpurun_out/sq_$TAG/$W
mkdir -p $D
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU"
P2="SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P -d $D/p$i -o run --output-format csv -- python bench.py --workload $W --steps 20 --warmup 5 --no-cpu-baseline > /dev/null
done
python tools/sq.py ${3:-k_env} $D/p1 $D/p2 | tail -3

#!/bin/bash
# Interleaved A/B of the reset-time ring fill (k_qfill) with the tuning build: per-launch kernel time
# over the first 80 launches after a reset, fill off / on, 3 reps.  Output: gpurun_out/<tag>/qfill_ab.log
O=gpurun_out/$1; mkdir -p $O
export PGTG_LIB=$PWD/pgtg_amd/libpgtg_hip_tuning.so
for rep in 1 2 3; do
  for q in 0 1; do
    PGTG_QFILL=$q timeout -k 10 120 python tools/ramp.py cfg5 80 > $O/ramp_q$q.log 2>&1 || exit 1
    echo "qfill=$q rep $rep: $(tail -5 $O/ramp_q$q.log | tr '\n' ' ')"
  done
done

#!/bin/bash
# A/B of the step kernels on one box (tuning build): k_envq (PGTG_PERSIST=0), k_envp with one helper
# wave, k_envp with two (PGTG_HELPERS=2); 3 interleaved reps of the driver's command shape and of a
# 400-step window.  Usage: bash tools/persist_ab.sh <tag> [workload]
O=gpurun_out/$1; W=${2:-cfg5}; mkdir -p $O
export PGTG_LIB=$PWD/pgtg_amd/libpgtg_hip_tuning.so
for rep in 1 2 3; do
  for v in q p1 p2; do
    case $v in q) P=0; H=1 ;; p1) P=1; H=1 ;; p2) P=1; H=2 ;; esac
    PGTG_PERSIST=$P PGTG_HELPERS=$H timeout -k 10 120 python bench.py --workload $W --steps 20 --warmup 5 --no-cpu-baseline > $O/$v.json 2> $O/$v.err || { tail -5 $O/$v.err; exit 1; }
    PGTG_PERSIST=$P PGTG_HELPERS=$H timeout -k 10 120 python bench.py --workload $W --steps 400 --warmup 50 --no-cpu-baseline > $O/l$v.json 2> $O/l$v.err || { tail -5 $O/l$v.err; exit 1; }
    python -c "
import json
for f in ('$O/$v.json', '$O/l$v.json'):
    d=json.load(open(f)); r=d['roofline']
    print('$v rep $rep', r['kernel'][:18], d['steps'], 'steps:', f\"{d['value']/1e9:.3f} G, {d['ms_per_step']*1e3:.1f} us/step, kern {r['avg_kernel_us']:.1f} us\")"
  done
done

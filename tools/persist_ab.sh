#!/bin/bash
# A/B of the persistent step kernel (k_envp) against k_envq on one box (tuning build, PGTG_PERSIST=0/1),
# 3 interleaved reps of the driver's own command shape and of a 400-step window.
O=gpurun_out/$1; W=${2:-cfg5}; mkdir -p $O
export PGTG_LIB=$PWD/pgtg_amd/libpgtg_hip_tuning.so
for rep in 1 2 3; do
  for p in 0 1; do
    PGTG_PERSIST=$p timeout -k 10 120 python bench.py --workload $W --steps 20 --warmup 5 --no-cpu-baseline > $O/p$p.json 2> $O/p$p.err || { tail -5 $O/p$p.err; exit 1; }
    PGTG_PERSIST=$p timeout -k 10 120 python bench.py --workload $W --steps 400 --warmup 50 --no-cpu-baseline > $O/pl$p.json 2> $O/pl$p.err || { tail -5 $O/pl$p.err; exit 1; }
    python -c "
import json
for f in ('$O/p$p.json', '$O/pl$p.json'):
    d=json.load(open(f)); r=d['roofline']
    print('persist=$p rep $rep', r['kernel'][:18], d['steps'], 'steps:', f\"{d['value']/1e9:.3f} G, {d['ms_per_step']*1e3:.1f} us/step, kern {r['avg_kernel_us']:.1f} us\")"
  done
done

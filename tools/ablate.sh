#!/bin/bash
# k_envq ablations (tuning build, PGTG_ABL bits: 1 no ring refills, 2 no terminal writes, 4 no
# observation writes): kernel time per launch of each, interleaved, 2 reps.  Results of ablated runs
# are wrong by construction; only the timing is read.  Usage: bash tools/ablate.sh <tag> [workload]
O=gpurun_out/$1; W=${2:-cfg5}; mkdir -p $O
export PGTG_LIB=$PWD/pgtg_amd/libpgtg_hip_tuning.so
for rep in 1 2; do
  for a in 0 1 2 4 6 7; do
    PGTG_ABL=$a timeout -k 10 120 python bench.py --workload $W --steps 200 --warmup 20 --no-cpu-baseline > $O/abl_$a.json 2> $O/abl_$a.err || { tail -5 $O/abl_$a.err; exit 1; }
    python -c "import json; d=json.load(open('$O/abl_$a.json')); r=d['roofline']; print('abl=$a rep $rep', f\"kern {r['avg_kernel_us']:.1f}us\")"
  done
done

#!/bin/bash
# round 5 session 5: env-wave priority A/B (configs[4]); shard-size launch shapes (64/32-env workgroups)
set -o pipefail
O=gpurun_out/r05s5; mkdir -p $O
AB_STEPS=200 timeout -k 10 600 bash tools/ab_multi.sh cfg5 3 new ab/prio1.so ab/prio2.so > $O/ab_prio.log 2>&1 || { cat $O/ab_prio.log; exit 1; }
grep -v amdgpu.ids $O/ab_prio.log
for n in 131072 262144; do
  for epb in 0 64 32; do
    timeout -k 10 120 python bench.py --envs $n --envs-per-block $epb --steps 400 --warmup 50 --no-cpu-baseline > $O/shard_${n}_$epb.json 2> $O/shard_${n}_$epb.err || { tail $O/shard_${n}_$epb.err; exit 1; }
    python -c "import json; d=json.load(open('$O/shard_${n}_$epb.json')); r=d['roofline']; print('$n epb=$epb', f\"{d['value']/1e9:.3f}G\", f\"kern {r['avg_kernel_us']:.1f}us\", r['envs_per_workgroup'])"
  done
done

#!/bin/bash
# Interleaved A/B runs on one box.  Usage: bash tools/ab_multi.sh <workload> <reps> <variant>...
# A variant is a library -- a path to a .so, or "new" for the in-tree build -- optionally followed by
# settings separated by colons: ENV=VALUE (read by the tuning build, pgtg_amd/build.py TOOL_VARIANTS)
# or --bench-option=VALUE, e.g.
#   pgtg_amd/libpgtg_hip_tuning.so:PGTG_ABL=1      k_envq ablation (1 no ring refills, 2 no terminal
#                                                   writes, 4 no observation writes; timing only)
#   new:--kt-wpc=2                                 k_traffic workgroups per CU
#   new:--envs-per-block=64:--envs=131072          launch shape at a shard size
#   ab/old.so:PGTG_ABI_COMPAT=6:--envs=131072       a build of an older ABI version (pgtg_amd/_abi.py)
# Modes (environment): AB_STEPS / AB_WARMUP the bench window (100 / 20); AB_KTRACE=1 per-kernel
# rocprofv3 averages (k_env, k_traffic separately) instead of the bench line; AB_RAMP=1 the
# per-launch kernel time of the first 80 launches after a reset (tools/ramp.py) instead.
W=$1; R=$2; shift 2
O=gpurun_out/ab; mkdir -p $O
export TMPDIR=/tmp
for rep in $(seq $R); do
  for V in "$@"; do
    IFS=: read -r L REST <<< "$V"
    (
      if [ "$L" = new ]; then unset PGTG_LIB; else export PGTG_LIB=$PWD/$L; fi
      ARGS=()
      IFS=: read -ra SET <<< "$REST"
      for s in "${SET[@]}"; do
        case $s in
          --*) ARGS+=("${s%%=*}" "${s#*=}") ;;
          *=*) export "$s" ;;
        esac
      done
      if [ "${AB_RAMP:-0}" = 1 ]; then
        timeout -k 10 120 python tools/ramp.py $W 80 > $O/ramp.log 2>&1 || { tail -5 $O/ramp.log; exit 1; }
        echo "$V rep $rep: $(tail -5 $O/ramp.log | tr '\n' ' ')"
      elif [ "${AB_KTRACE:-0}" = 1 ]; then
        rm -rf $O/kt
        timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- python bench.py --workload $W --steps ${AB_STEPS:-400} --warmup ${AB_WARMUP:-200} --no-cpu-baseline "${ARGS[@]}" > $O/kt.json 2> $O/kt.err || { tail -5 $O/kt.err; exit 1; }
        f=$(find $O/kt -name "*kernel_stats.csv" | head -1)
        python -c "
import csv
print('$W $V', '  '.join(f\"{r['Name'][:18]} {float(r['AverageNs'])/1e3:.1f}us\" for r in csv.DictReader(open('$f')) if 'k_env' in r['Name'] or 'k_traffic' in r['Name']))"
      else
        timeout -k 10 180 python bench.py --workload $W --steps ${AB_STEPS:-100} --warmup ${AB_WARMUP:-20} --no-cpu-baseline "${ARGS[@]}" > $O/abm.json 2> $O/abm.err || { tail -5 $O/abm.err; exit 1; }
        python -c "import json; d=json.load(open('$O/abm.json')); r=d['roofline']; print('$W $V', f\"{d['value']/1e6:.2f}M\", f\"kern {r['avg_kernel_us']:.1f}us\")"
      fi
    ) || exit 1
  done
done

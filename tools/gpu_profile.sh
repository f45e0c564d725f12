#!/bin/bash
# One GPU session of measurements for DESIGN.md / profiles/: per workload a bench line, a
# rocprofv3 kernel-trace summary and the two PMC passes (FETCH_SIZE, WRITE_SIZE) that give
# roofline.traffic.  Usage: bash tools/gpu_profile.sh <tag> [workloads...]
# The trace runs the bench's own window (50 warm-up + 1000 timed steps), so its kernel average is the
# one the bench line's events measure; the PMC passes profile the steps after a 200-step warm-up (the
# median is taken over the dispatches after the first 10), the steady state that dominates that window
# (the first steps after a common reset regenerate 25-45 % of the traffic envs at once).
set -e
TAG=${1:-dev}
shift || true
WLS=${@:-cfg2 cfg4 cfg5 cfg3}
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_$TAG
python -c "from pgtg_amd.build import build; build()" || exit 1
for W in $WLS; do
  D=gpurun_out/prof_$TAG/$W
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/trace -o run --output-format csv -- python bench.py --workload $W --steps 1000 --warmup 50 --no-cpu-baseline > $D.trace.json
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $D/fetch -o run --output-format csv -- python bench.py --workload $W --steps 60 --warmup 200 --no-cpu-baseline > /dev/null
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $D/write -o run --output-format csv -- python bench.py --workload $W --steps 60 --warmup 200 --no-cpu-baseline > /dev/null
  python tools/pmc.py $W $D/fetch $D/write $TAG > $D.pmc.json
  cp profiles/pmc_$W.json $D.pmc_profile.json
  timeout -k 10 300 python bench.py --workload $W --no-cpu-baseline > $D.bench.json
  echo "$W done"
done

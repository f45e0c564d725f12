#!/bin/bash
# One GPU session of measurements for DESIGN.md / profiles/: per workload a bench line, a
# rocprofv3 kernel-trace summary and the two PMC passes (FETCH_SIZE, WRITE_SIZE) that give
# roofline.traffic.  Usage: bash tools/gpu_profile.sh <tag> [workloads...]
set -e
TAG=${1:-dev}
shift || true
WLS=${@:-cfg2 cfg4 cfg5 cfg3}
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_$TAG
python -c "from pgtg_amd.build import build; build()" || exit 1
for W in $WLS; do
  D=gpurun_out/prof_$TAG/$W
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/trace -o run --output-format csv -- python bench.py --workload $W --steps 100 --warmup 20 --no-cpu-baseline > $D.trace.json
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $D/fetch -o run --output-format csv -- python bench.py --workload $W --steps 40 --warmup 10 --no-cpu-baseline > /dev/null
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $D/write -o run --output-format csv -- python bench.py --workload $W --steps 40 --warmup 10 --no-cpu-baseline > /dev/null
  python tools/pmc.py $W $D/fetch $D/write $TAG > $D.pmc.json
  cp profiles/pmc_$W.json $D.pmc_profile.json
  timeout -k 10 300 python bench.py --workload $W --steps 200 --warmup 20 --no-cpu-baseline > $D.bench.json
  echo "$W done"
done

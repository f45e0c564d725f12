#!/bin/bash
# Round-2 GPU session 3: PMC calibration, rule-layout tests, launch-shape A/B, profiles of cfg5 (the
# default line at 1 048 576 envs) and cfg3.
set -o pipefail
O=gpurun_out/r02s3
mkdir -p $O
export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE -d $O/calib_fetch -o run --output-format csv -- ./tools/micro/pmc_calib > $O/calib.log 2>&1 || exit 1
timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE -d $O/calib_write -o run --output-format csv -- ./tools/micro/pmc_calib >> $O/calib.log 2>&1 || exit 1
python tools/pmc_calib.py $O/calib_fetch $O/calib_write > $O/calib.json || exit 1
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_env.py > $O/env_tests.log 2>&1; echo "env tests rc=$?"; tail -3 $O/env_tests.log
for W in cfg4 cfg2 cfg3; do
  timeout -k 10 300 python -u bench.py --workload $W --steps 200 --warmup 20 --no-cpu-baseline > $O/b_$W.json || exit 1
done
timeout -k 10 300 python -u bench.py --workload cfg4 --steps 200 --warmup 20 --no-cpu-baseline --envs-per-block 256 > $O/b_cfg4_wg256.json || exit 1
timeout -k 10 900 bash tools/gpu_profile.sh r02s3 cfg5 cfg3 > $O/profile.log 2>&1; echo "profile rc=$?"
cp -r gpurun_out/prof_r02s3 $O/ 2>/dev/null
python - <<'PY'
import json,glob
for f in sorted(glob.glob("gpurun_out/r02s3/b_*.json")):
    d=json.loads(open(f).read().strip().splitlines()[-1]); r=d["roofline"]
    print(f, f"{d['value']/1e6:.1f}M", f"{r['avg_kernel_us']:.1f}us", r["kernel"], f"frac {r['frac']:.3f}", f"peak {r['peak']:.0f}")
PY
cat $O/calib.json

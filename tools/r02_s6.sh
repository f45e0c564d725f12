#!/bin/bash
# Quick traffic check: car-store parity + the cfg3 bench line (optionally a kernel-stats profile).
set -o pipefail
O=gpurun_out/${TAG:-r02s6}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_car_slots.py tests/test_gpu_parity.py tests/test_gpu_occupancy.py "tests/test_gpu_exhaustive.py::test_cfg3_long_cautious_traffic" "tests/test_gpu_exhaustive.py::test_every_env_every_step[cfg3_all_65536x3]" > $O/pytest_traffic.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_traffic.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u bench.py --workload cfg3 --steps 200 --warmup 20 --no-cpu-baseline > $O/b_cfg3.json || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python bench.py --workload cfg3 --steps 100 --warmup 20 --no-cpu-baseline > $O/trace.json || exit 1
python - <<'PY'
import csv, glob, json, os
O = os.environ.get("TAG", "r02s6")
d = json.loads(open(f"gpurun_out/{O}/b_cfg3.json").read().strip().splitlines()[-1])
print("cfg3", f"{d['value']/1e6:.2f}M env-steps/s", f"{d['roofline']['avg_kernel_us']:.1f} us")
for f in glob.glob(f"gpurun_out/{O}/trace/**/run_kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "k_env" in r["Name"] or "k_traffic" in r["Name"]:
            print(r["Name"][:28], r["Calls"], float(r["AverageNs"]) / 1e3)
PY

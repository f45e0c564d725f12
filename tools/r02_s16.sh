#!/bin/bash
# Single-bank car store, final form: traffic parity, then the cfg3 profile (bench, kernel stats, PMC).
set -o pipefail
O=gpurun_out/r02s16
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_car_slots.py tests/test_gpu_parity.py tests/test_gpu_occupancy.py tests/test_gpu_traffic_groups.py tests/test_gpu_exhaustive.py tests/test_gpu_state.py tests/test_gpu_env.py tests/test_gpu_vec.py tests/test_gpu_config_fuzz.py tests/test_gpu_bench_sizes.py > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 900 bash tools/gpu_profile.sh r02s16 cfg3 > $O/profile.log 2>&1; echo "profile rc=$?"
cp -r gpurun_out/prof_r02s16 $O/ 2>/dev/null
cat $O/prof_r02s16/cfg3.bench.json; cat $O/prof_r02s16/cfg3.pmc.json

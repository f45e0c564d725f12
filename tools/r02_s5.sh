#!/bin/bash
# Round-2 GPU session 5: single-bank car store -- traffic parity (golden trajectories, exhaustive
# cfg3, car-slot compaction, saturating counters), then cfg3 bench + kernel stats + PMC traffic.
set -o pipefail
O=gpurun_out/r02s5
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_car_slots.py tests/test_gpu_parity.py tests/test_gpu_occupancy.py tests/test_gpu_traffic_groups.py "tests/test_gpu_exhaustive.py::test_cfg3_long_cautious_traffic" "tests/test_gpu_exhaustive.py::test_every_env_every_step[cfg3_all_65536x3]" "tests/test_gpu_exhaustive.py::test_every_env_every_step[sliding_traffic_6000]" tests/test_gpu_state.py tests/test_gpu_env.py > $O/pytest_traffic.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 $O/pytest_traffic.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u bench.py --workload cfg3 --steps 200 --warmup 20 --no-cpu-baseline > $O/b_cfg3.json || exit 1
timeout -k 10 900 bash tools/gpu_profile.sh r02s5 cfg3 > $O/profile.log 2>&1; echo "profile rc=$?"
cp -r gpurun_out/prof_r02s5 $O/ 2>/dev/null
cat $O/b_cfg3.json

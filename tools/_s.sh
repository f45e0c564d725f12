set -o pipefail
O=gpurun_out/r06s1; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 60 ./tools/micro/hwid3 > $O/hwid3.log 2>&1; grep -v amdgpu.ids $O/hwid3.log
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_faults.py tests/test_gpu_vec.py tests/test_gpu_exhaustive.py -k "fault or flat or sb3 or one_round" > $O/pytest_new.log 2>&1
rc=$?; tail -15 $O/pytest_new.log; [ $rc = 0 ] || exit 1
AB_STEPS=400 AB_WARMUP=30 timeout -k 10 900 bash tools/ab_multi.sh cfg5 2 new:--envs=131072 ab/r05_pre_persist.so:PGTG_ABI_COMPAT=6:--envs=131072 pgtg_amd/libpgtg_hip_tuning.so:PGTG_ABL=1:--envs=131072 pgtg_amd/libpgtg_hip_tuning.so:PGTG_ABL=6:--envs=131072 pgtg_amd/libpgtg_hip_tuning.so:PGTG_ABL=16:--envs=131072 new:--envs=262144 ab/r05_pre_persist.so:PGTG_ABI_COMPAT=6:--envs=262144 > $O/ab.log 2>&1 || { cat $O/ab.log; exit 1; }
grep -v amdgpu.ids $O/ab.log
timeout -k 10 300 python tools/stamps.py cfg5 > $O/stamps.log 2>&1 || { tail -20 $O/stamps.log; exit 1; }
cat $O/stamps.log

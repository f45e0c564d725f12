set -o pipefail
O=gpurun_out/r06s4; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_vec.py tests/test_gpu_faults.py > $O/pytest.log 2>&1
rc=$?; tail -4 $O/pytest.log; [ $rc = 0 ] || exit 1
bash tools/gpu_session.sh r06s4 adapter || exit 1
T=pgtg_amd/libpgtg_hip_tuning.so
AB_STEPS=400 AB_WARMUP=30 timeout -k 10 900 bash tools/ab_multi.sh cfg5 2 new:--envs=131072 $T:PGTG_ABL=128:--envs=131072 new:--envs=262144 $T:PGTG_ABL=128:--envs=262144 > $O/ab.log 2>&1 || { cat $O/ab.log; exit 1; }
grep -v amdgpu.ids $O/ab.log
bash tools/gpu_session.sh r06s4 ranks

set -o pipefail
O=gpurun_out/r06s3; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -4 $O/pytest.log; [ $rc = 0 ] || exit 1
T=pgtg_amd/libpgtg_hip_tuning.so
AB_STEPS=400 AB_WARMUP=30 timeout -k 10 900 bash tools/ab_multi.sh cfg5 2 new:--envs=131072 new:--envs=131072:--queue-mode=1 ab/r05_pre_persist.so:PGTG_ABI_COMPAT=6:--envs=131072 $T:PGTG_PRIO=2:--envs=131072 $T:PGTG_QPAD=0:PGTG_PPAD=0:--envs=131072 new:--envs=262144 new:--envs=262144:--queue-mode=1 new:--envs=524288 new:--envs=524288:--queue-mode=2 > $O/ab.log 2>&1 || { cat $O/ab.log; exit 1; }
grep -v amdgpu.ids $O/ab.log
AB_STEPS=1000 AB_WARMUP=50 timeout -k 10 900 bash tools/ab_multi.sh cfg2 3 new new:--queue-mode=1 $T:PGTG_PRIO=2 > $O/abcfg2.log 2>&1 || { cat $O/abcfg2.log; exit 1; }
grep -v amdgpu.ids $O/abcfg2.log
timeout -k 10 300 python tools/stamps.py cfg5 > $O/stamps_b.log 2>&1 || { tail -20 $O/stamps_b.log; exit 1; }
cat $O/stamps_b.log
bash tools/gpu_session.sh r06s3 adapter

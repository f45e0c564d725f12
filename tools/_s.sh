set -o pipefail
O=gpurun_out/r06s2; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -4 $O/pytest.log; [ $rc = 0 ] || exit 1
T=pgtg_amd/libpgtg_hip_tuning.so
AB_STEPS=400 AB_WARMUP=30 timeout -k 10 900 bash tools/ab_multi.sh cfg5 2 new:--envs=131072 $T:PGTG_ABL=64:--envs=131072 ab/r05_pre_persist.so:PGTG_ABI_COMPAT=6:--envs=131072 $T:PGTG_QPAD=0:PGTG_PPAD=0:--envs=131072 $T:PGTG_ABL=64:PGTG_QPAD=0:PGTG_PPAD=0:--envs=131072 > $O/ab131k.log 2>&1 || { cat $O/ab131k.log; exit 1; }
grep -v amdgpu.ids $O/ab131k.log
AB_STEPS=400 AB_WARMUP=30 timeout -k 10 900 bash tools/ab_multi.sh cfg5 2 new:--envs=262144 $T:PGTG_ABL=64:--envs=262144 ab/r05_pre_persist.so:PGTG_ABI_COMPAT=6:--envs=262144 new:--envs=524288 $T:PGTG_ABL=64:--envs=524288 > $O/ab262k.log 2>&1 || { cat $O/ab262k.log; exit 1; }
grep -v amdgpu.ids $O/ab262k.log
AB_STEPS=200 AB_WARMUP=30 timeout -k 10 900 bash tools/ab_multi.sh cfg5 2 new $T:PGTG_ABL=64 ab/r05_pre_persist.so:PGTG_ABI_COMPAT=6 > $O/ab1m.log 2>&1 || { cat $O/ab1m.log; exit 1; }
grep -v amdgpu.ids $O/ab1m.log
AB_STEPS=1000 AB_WARMUP=50 timeout -k 10 900 bash tools/ab_multi.sh cfg2 3 new $T:PGTG_ABL=64 ab/r05_pre_persist.so:PGTG_ABI_COMPAT=6 > $O/abcfg2.log 2>&1 || { cat $O/abcfg2.log; exit 1; }
grep -v amdgpu.ids $O/abcfg2.log
timeout -k 10 300 python tools/stamps.py cfg5 > $O/stamps_new.log 2>&1 || { tail -20 $O/stamps_new.log; exit 1; }
cat $O/stamps_new.log
PGTG_ABI_COMPAT=6 PGTG_STAMPS_LIB=$PWD/ab/r05_pre_persist_stamps.so timeout -k 10 300 python tools/stamps.py cfg5 > $O/stamps_old.log 2>&1 || { tail -20 $O/stamps_old.log; exit 1; }
cat $O/stamps_old.log

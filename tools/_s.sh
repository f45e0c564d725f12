set -o pipefail
O=gpurun_out/r06s18; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_vec.py > $O/pytest_q.log 2>&1
rc=$?; tail -5 $O/pytest_q.log; [ $rc = 0 ] || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/adp -o run --output-format csv -- python bench.py --adapter device --steps 100 --warmup 20 > $O/adp.json 2> $O/adp.err || { tail $O/adp.err; exit 1; }
f=$(find $O/adp -name "*kernel_stats.csv" | head -1); cut -d, -f2-4 $f | head -6
bash tools/gpu_session.sh r06s18 adapter

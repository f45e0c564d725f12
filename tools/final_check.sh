#!/bin/bash
# Round-end style check of the committed tree on one GPU: GPU tests, smoke(), the default bench
# line (with the CPU baseline) and a fresh profile of the bench workload.  Usage: bash tools/final_check.sh <tag>
TAG=${1:-final}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
tail -2 gpurun_out/${TAG}_tests.log
grep -q " passed" gpurun_out/${TAG}_tests.log && ! grep -q "failed\|error" gpurun_out/${TAG}_tests.log || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || exit 1
tail -1 gpurun_out/${TAG}_smoke.log
timeout -k 10 300 python bench.py > gpurun_out/${TAG}_bench_default.json 2> gpurun_out/${TAG}_bench_default.err || exit 1
cat gpurun_out/${TAG}_bench_default.json
bash tools/gpu_profile.sh $TAG cfg5 > gpurun_out/${TAG}_prof.log 2>&1 || exit 1
echo profile done

#!/bin/bash
# Round-2 GPU session 1: configs[4] at its full 1 048 576 envs on one GPU (default line and the
# 128-env map-queue launch shape), the two-rank digest rehearsal, then the GPU test suite.
set -o pipefail
O=gpurun_out/r02s1
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --steps 200 --warmup 30 > $O/b_default.json 2> $O/b_default.err || exit 1
PGTG_ENVS_PER_BLOCK=128 timeout -k 10 300 python -u bench.py --steps 200 --warmup 30 --no-cpu-baseline > $O/b_epb128.json 2> $O/b_epb128.err || exit 1
timeout -k 10 200 python -u bench.py --envs 131072 --steps 20 --warmup 5 --no-cpu-baseline --digest $O/dg1 > $O/dg1.json 2>&1 || exit 1
PGTG_BENCH_SAME_GPU=1 PGTG_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --envs 131072 --steps 20 --warmup 5 --digest $O/dg2 > $O/dg2.json 2> $O/dg2.err || exit 1
python tools/digest_compare.py $O/dg1 $O/dg2 > $O/digest_compare.json
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
echo "pytest rc=$?"
tail -3 $O/pytest_gpu.log
cat $O/b_default.json $O/b_epb128.json $O/digest_compare.json

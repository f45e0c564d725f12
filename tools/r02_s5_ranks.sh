#!/bin/bash
# Sharded-path rehearsal on a one-GPU lease at the full configs[4] batch (1 048 576 envs): a
# single-process run and 2- and 4-rank torch.distributed runs (gloo, all ranks on GPU 0) save
# per-env output digests after the timed window; every rank's slice must equal the single run's.
set -o pipefail
O=gpurun_out/r02s5r
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --steps 40 --warmup 10 --no-cpu-baseline --digest $O/dg1 > $O/dg1.json 2> $O/dg1.err || exit 1
for N in 2 4; do
  PGTG_BENCH_SAME_GPU=1 PGTG_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N \
    --master-addr 127.0.0.1 --master-port 2951$N bench.py --gpus $N --steps 40 --warmup 10 --digest $O/dg$N > $O/dg$N.json 2> $O/dg$N.err || exit 1
  python tools/digest_compare.py $O/dg1 $O/dg$N > $O/digest_compare_$N.json || exit 1
done
rm -f $O/*.npz  # 64 MB each: keep gpurun_out small enough to travel back
cat $O/dg1.json $O/dg2.json $O/dg4.json $O/digest_compare_2.json $O/digest_compare_4.json

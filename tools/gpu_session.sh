#!/bin/bash
# One GPU call made of named steps, each under its own time limit; the first failing step ends the
# call.  Output under gpurun_out/<tag>/.  Usage: bash tools/gpu_session.sh <tag> <step>...
#   tests            pytest -m gpu (whole suite)
#   tests:<expr>     pytest -m gpu -k <expr>
#   smoke            __graft_entry__.smoke()
#   bench            the default bench line (configs[4], with the CPU baseline)
#   driver           the driver's own line: bench.py --gpus 1 --steps 20 --warmup 5
#   ramp:<wl>        per-launch kernel time of the first 80 launches after a reset (tools/ramp.py)
#   bench:<wl>       bench.py --workload <wl> --steps 200 --warmup 20
#   benchlong:<wl>   bench.py --workload <wl> with the default 1000-step window
#   rccl             bench.py under torch.distributed.run, one rank, nccl backend, --dist (RCCL init +
#                    the device counter all-reduce), 131 072 envs
#   ranks            2, 4 and 8 ranks on one GPU (gloo) at the full configs[4] batch (8 ranks: the 131 072-env
#                    one-round shard of an 8-GPU run), per-env digests vs one process
#   shards           single-process lines at the per-rank shards of N = 2, 4, 8 (524 288 / 262 144 /
#                    131 072 envs) beside the 1 048 576-env line
#   adapter          bench.py --adapter device / host / host-monitor (the SB3 VecEnv adapter, caller workload)
#   hwid3            wave-to-SIMD placement of four resident 256-thread workgroups per CU (tools/micro/hwid3)
#   profile:<wl,..>  tools/gpu_profile.sh (rocprofv3 kernel stats + FETCH_SIZE / WRITE_SIZE passes)
#   genbench         map-generation latency per map (tools/genbench.py, stamps build)
#   stamps:<wl,..>   per-phase cycle stamps (PGTG_STAMPS build, tools/stamps.py)
#   stampsjson:<wl> the latency record bench.py reads (copy gpurun_out/<tag>/stamps_<wl>.json to profiles/)
#   stampslib:<lib>:<wl>  the same with a prebuilt stamps library
#   ab:<wl>:<lib>    interleaved bench lines of the in-tree library and <lib> (tools/ab_multi.sh, 3 reps)
#   libtests:<lib>:<expr>  pytest -m gpu -k <expr> against another build of the library (PGTG_LIB)
#   pmc:<wl>:<lib|new>     FETCH_SIZE / WRITE_SIZE passes of one workload with a given library
#   sq:<wl>          SQ instruction/stall passes of one workload -> gpurun_out/<tag>/sq_<wl>.json (issue roofline)
# Round-end records (profiles/r06/final) came from three calls:
#   tests smoke bench driver benchlong:cfg2 benchlong:cfg3 benchlong:cfg4 benchlong:train shards rccl
#   profile:cfg5,cfg2 stampsjson:cfg2 adapter ranks
#   tests smoke bench driver adapter            (after the last k_flatten change)
set -o pipefail
TAG=$1
shift
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
for S in "$@"; do
  echo "== $S $(date +%T)"
  case $S in
    tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $O/pytest.log 2>&1
      rc=$?; tail -3 $O/pytest.log; [ $rc = 0 ] || exit 1 ;;
    tests:*)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread -k "${S#tests:}" > $O/pytest_k.log 2>&1
      rc=$?; tail -5 $O/pytest_k.log; [ $rc = 0 ] || exit 1 ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
      tail -2 $O/smoke.log ;;
    bench)
      timeout -k 10 400 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
      cat $O/bench_default.json ;;
    driver)
      timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err || { tail -20 $O/bench_driver.err; exit 1; }
      python tools/bench_line.py $O/bench_driver.json ;;
    ramp:*)
      timeout -k 10 300 python -u tools/ramp.py ${S#ramp:} > $O/ramp_${S#ramp:}.log 2>&1 || { tail -20 $O/ramp_${S#ramp:}.log; exit 1; }
      tail -6 $O/ramp_${S#ramp:}.log ;;
    benchlong:*)
      W=${S#benchlong:}
      timeout -k 10 400 python -u bench.py --workload $W --no-cpu-baseline > $O/benchlong_$W.json 2> $O/benchlong_$W.err || { tail -20 $O/benchlong_$W.err; exit 1; }
      python tools/bench_line.py $O/benchlong_$W.json ;;
    bench:*)
      W=${S#bench:}
      timeout -k 10 300 python -u bench.py --workload $W --steps 200 --warmup 20 --no-cpu-baseline > $O/bench_$W.json 2> $O/bench_$W.err || { tail -20 $O/bench_$W.err; exit 1; }
      python tools/bench_line.py $O/bench_$W.json ;;
    rccl)
      timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
        --master-port 29517 bench.py --dist --envs 131072 --steps 200 --warmup 20 --no-cpu-baseline \
        > $O/rccl.json 2> $O/rccl.err || { tail -30 $O/rccl.err; exit 1; }
      cat $O/rccl.json ;;
    ranks)
      # the sharded path rehearsed on one GPU: 2 and 4 ranks (gloo counters, every rank on GPU 0) at the full
      # configs[4] batch; every rank's per-env output digests against the single-process run's
      timeout -k 10 300 python -u bench.py --steps 30 --warmup 10 --no-cpu-baseline --digest $O/dg1 > $O/ranks_1.json 2> $O/ranks_1.err || { tail -20 $O/ranks_1.err; exit 1; }
      for N in 2 4 8; do
        PGTG_BENCH_SAME_GPU=1 PGTG_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 \
          --nproc-per-node $N --master-addr 127.0.0.1 --master-port $((29600 + N)) bench.py --gpus $N --steps 30 \
          --warmup 10 --no-cpu-baseline --digest $O/dg$N > $O/ranks_$N.json 2> $O/ranks_$N.err || { tail -30 $O/ranks_$N.err; exit 1; }
        python tools/digest_compare.py $O/dg1 $O/dg$N | tee $O/digest_compare_$N.json || exit 1
      done
      rm -f $O/dg*.npz ;;  # (64 MB each: gpurun returns at most 64 MiB)
    shards)
      for N in 1048576 524288 262144 131072; do
        timeout -k 10 300 python -u bench.py --envs $N --steps 400 --warmup 30 --no-cpu-baseline > $O/shard_$N.json 2> $O/shard_$N.err || { tail -20 $O/shard_$N.err; exit 1; }
        python tools/bench_line.py $O/shard_$N.json
      done ;;
    adapter)
      for M in device host host-monitor; do
        timeout -k 10 300 python -u bench.py --adapter $M --steps 200 --warmup 20 > $O/adapter_$M.json 2> $O/adapter_$M.err || { tail -20 $O/adapter_$M.err; exit 1; }
        python -c "import json; d=json.load(open('$O/adapter_$M.json')); print('$M', round(d['value'] / 1e6, 2), 'M env-steps/s', round(d['ms_per_step'], 2), 'ms/step')"
      done ;;
    hwid3)
      timeout -k 10 60 ./tools/micro/hwid3 > $O/hwid3.log 2>&1 || { tail -20 $O/hwid3.log; exit 1; }
      grep -v amdgpu.ids $O/hwid3.log ;;
    profile:*)
      R=${S#profile:}; timeout -k 10 1500 bash tools/gpu_profile.sh $TAG ${R//,/ } > $O/profile.log 2>&1 || { tail -20 $O/profile.log; exit 1; }
      tail -5 $O/profile.log ;;
    genbench)
      timeout -k 10 120 python tools/genbench.py 5 1024 8 > $O/genbench.log 2>&1 || { tail -20 $O/genbench.log; exit 1; }
      tail -1 $O/genbench.log ;;
    stamps:*)
      python -c "from pgtg_amd.build import build; build(variant='stamps')" || exit 1
      R=${S#stamps:}; timeout -k 10 300 python tools/stamps.py ${R//,/ } > $O/stamps.log 2>&1 || { tail -20 $O/stamps.log; exit 1; }
      cat $O/stamps.log ;;
    stampsjson:*)
      W=${S#stampsjson:}
      PGTG_STAMPS_JSON=$O/stamps_$W.json PGTG_STAMPS_WL=$W timeout -k 10 300 python tools/stamps.py $W > $O/stampsjson_$W.log 2>&1 || { tail -20 $O/stampsjson_$W.log; exit 1; }
      cat $O/stamps_$W.json ;;
    stampslib:*)
      R=${S#stampslib:}; L=${R%%:*}; W=${R#*:}
      PGTG_STAMPS_LIB=$PWD/$L timeout -k 10 300 python tools/stamps.py $W > $O/stamps_$(basename $L .so).log 2>&1 || { tail -20 $O/stamps_$(basename $L .so).log; exit 1; }
      cat $O/stamps_$(basename $L .so).log ;;
    libtests:*)
      R=${S#libtests:}; L=${R%%:*}; K=${R#*:}
      PGTG_LIB=$PWD/$L timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread -k "$K" > $O/pytest_lib.log 2>&1
      rc=$?; tail -3 $O/pytest_lib.log; [ $rc = 0 ] || exit 1 ;;
    pmc:*)
      R=${S#pmc:}; W=${R%%:*}; L=${R#*:}; N=$(basename $L .so)
      D=$O/pmc_${W}_$N
      if [ $L = new ]; then unset PGTG_LIB; else export PGTG_LIB=$PWD/$L; fi
      timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $D/fetch -o run --output-format csv -- python bench.py --workload $W --steps 60 --warmup 200 --no-cpu-baseline > /dev/null 2>$D.err || { tail $D.err; exit 1; }
      timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $D/write -o run --output-format csv -- python bench.py --workload $W --steps 60 --warmup 200 --no-cpu-baseline > /dev/null 2>>$D.err || { tail $D.err; exit 1; }
      unset PGTG_LIB
      python tools/pmc.py $W $D/fetch $D/write $N > $D.json || exit 1
      python -c "import json; d=json.load(open('$D.json')); print('$W $N', {k: round((v['read_bytes']+v['write_bytes'])/1e6,1) for k,v in d.items() if isinstance(v,dict)}, round(d['hbm_bytes_per_launch']/1e6,1), 'MB/launch')" ;;
    ab:*)
      R=${S#ab:}; W=${R%%:*}; L=${R#*:}
      timeout -k 10 900 bash tools/ab_multi.sh $W 3 new $L > $O/ab_$W.log 2>&1 || { tail -20 $O/ab_$W.log; exit 1; }
      cat $O/ab_$W.log ;;
    sq:*)
      W=${S#sq:}
      timeout -k 10 300 bash tools/sq_passes.sh $TAG $W > $O/sq_$W.log 2>&1 || { tail -20 $O/sq_$W.log; exit 1; }
      N=$(python -c "import bench; print(bench.WORKLOADS['$W'][2])")
      python tools/sq_json.py $W $N gpurun_out/sq_$TAG/$W/p1 gpurun_out/sq_$TAG/$W/p2 > $O/sq_$W.json || exit 1
      python tools/sq_summary.py k_ gpurun_out/sq_$TAG/$W/p1 gpurun_out/sq_$TAG/$W/p2 ;;
    *) echo "unknown step $S"; exit 2 ;;
  esac
done
echo "== done $(date +%T)"

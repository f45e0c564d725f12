#!/bin/bash
# Round 2, last session: the GPU suite, smoke() and the default bench line on the final tree, then an
# interleaved A/B of the timed loop (one pgtg_step host call per step vs one pgtg_step_many call).
O=gpurun_out/r02s5
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
tail -2 $O/tests.log
grep -q " passed" $O/tests.log && ! grep -q "failed\|error" $O/tests.log || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py > $O/default.json 2> $O/default.err || exit 1
cat $O/default.json
for r in 1 2; do
  for w in cfg2 cfg4 cfg5; do
    for m in "" "--per-step"; do
      timeout -k 10 200 python bench.py --workload $w --no-cpu-baseline $m > $O/ab_${w}_${r}${m}.json 2>> $O/ab.err || exit 1
      python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], sys.argv[3] or 'step_many', round(d['value']/1e6,1), 'M', round(d['ms_per_step']*1e3,2), 'us/step, kernel', round(d['roofline']['avg_kernel_us'],2))" $O/ab_${w}_${r}${m}.json $w "$m" | tee -a $O/ab_summary.txt
    done
  done
done

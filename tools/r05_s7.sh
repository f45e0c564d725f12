#!/bin/bash
# round 5 session 7: tile-algebra sliding-window images (k_env<true>) -- parity of every window path, A/B
set -o pipefail
O=gpurun_out/r05s7; mkdir -p $O
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_exhaustive.py tests/test_gpu_parity.py tests/test_gpu_config_fuzz.py tests/test_gpu_bench_sizes.py tests/test_gpu_vec.py -k "train or sliding or s4 or fuzz or random_config or window or feature or bench or vec or sb3 or shard or time_limit" > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; grep -E "FAILED" $O/pytest.log | head; [ $rc -le 1 ] || exit 1
AB_STEPS=100 AB_WARMUP=50 timeout -k 10 400 bash tools/ab_multi.sh train 2 ab/r04.so new > $O/ab_train.log 2>&1 || { cat $O/ab_train.log; exit 1; }
grep -v amdgpu.ids $O/ab_train.log
for m in device host host-monitor; do
  timeout -k 10 300 python bench.py --adapter $m --steps 50 --warmup 10 > $O/adapter_$m.json 2> $O/adapter_$m.err || { tail $O/adapter_$m.err; exit 1; }
  python -c "import json; d=json.load(open('$O/adapter_$m.json')); print('adapter $m', f\"{d['value']/1e6:.2f}M\", f\"{d['ms_per_step']:.2f} ms/step\")"
done

set -o pipefail
for rep in 1 2; do
for E in 0 256; do
  timeout -k 10 120 python bench.py --workload cfg3 --steps 100 --warmup 20 --no-cpu-baseline --envs-per-block $E > gpurun_out/e23.json || exit 1
  python -c "import json; d=json.load(open('gpurun_out/e23.json')); r=d['roofline']; print('cfg3 epb $E', f\"{d['value']/1e6:.2f}M\", f\"kern {r['avg_kernel_us']:.1f}us\", r['envs_per_workgroup'], r['lds_bytes'], r['workgroups_per_cu'])"
done
done
timeout -k 10 300 python -u -m pytest -x -q --timeout 300 tests/test_gpu_bench_sizes.py -k traffic 2>&1 | tail -2

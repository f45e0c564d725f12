set -e
for E in 16 32 64 128 256; do
  for W in cfg2 cfg4; do
    PGTG_ENVS_PER_BLOCK=$E timeout -k 10 120 python bench.py --workload $W --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/sw_${W}_$E.json
    python -c "import json; d=json.load(open('gpurun_out/sw_${W}_$E.json')); r=d['roofline']; print('$W E=$E', f\"{d['value']/1e6:.1f}M\", f\"{r['avg_kernel_us']:.1f}us\", r['envs_per_workgroup'], r['lds_bytes'])"
  done
done

"""One-line summary of a bench.py JSON line: python tools/bench_line.py <file>."""
import json
import sys

d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
print(f"{d['config']['workload'][:11]} envs {d['config']['envs_per_gpu']}: {d['value'] / 1e6:.1f} M env-steps/s, "
      f"{d['ms_per_step']:.4f} ms/step, kernel {r['avg_kernel_us']:.1f} us ({r['timed_launches']} launches), "
      f"{r['achieved']:.0f} GB/s alg, frac {r['frac']:.3f} (spec {r['frac_spec']:.3f}, copy {r.get('peak_copy_measured', 0):.0f} GB/s)")

#!/bin/bash
# Round-2 measurement pass on the final tree: the default bench line (configs[4], with the CPU
# baseline), then per workload a bench line, rocprofv3 kernel stats and the two PMC passes.
set -o pipefail
O=gpurun_out/r02fin
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py > $O/b_default.json 2> $O/b_default.err || exit 1
cat $O/b_default.json
timeout -k 10 1500 bash tools/gpu_profile.sh r02fin cfg5 cfg4 cfg2 cfg3 > $O/profile.log 2>&1 || exit 1
cp -r gpurun_out/prof_r02fin $O/
python - <<'PY'
import csv, glob, json
for w in ("cfg5", "cfg4", "cfg2", "cfg3"):
    d = json.loads(open(f"gpurun_out/prof_r02fin/{w}.bench.json").read().strip().splitlines()[-1]); r = d["roofline"]
    p = json.load(open(f"gpurun_out/prof_r02fin/{w}.pmc.json"))
    ks = {}
    for row in csv.DictReader(open(f"gpurun_out/prof_r02fin/{w}/trace/run_kernel_stats.csv")):
        if "k_env" in row["Name"] or "k_traffic" in row["Name"]:
            ks[row["Name"].split("(")[0][-22:]] = round(float(row["AverageNs"]) / 1e3, 1)
    print(w, f"{d['value']/1e6:.1f}M", f"events {r['avg_kernel_us']:.1f}us", ks, f"alg {r['alg_bytes_per_launch']/1e6:.1f}MB", f"pmc {p['hbm_bytes_per_launch']/1e6:.1f}MB", f"frac {r['frac']:.3f}")
PY

"""Turn rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE; separate runs) of a bench.py workload into
profiles/pmc_<workload>.json: HBM bytes per step launch of k_env (+ k_traffic when present).

Usage: python tools/pmc.py <workload> <fetch_run_dir> <write_run_dir> [tag]
gfx950 calibration (/opt/skills/guides/MI355X_MICROARCH.md, HBM section): FETCH_SIZE counts half of
the bytes of 16-B-per-lane streaming reads -- the way k_env reads its env records and tile plans --
so the read bytes are taken as 2 x FETCH_SIZE; WRITE_SIZE is taken as is.  Both counters report KB."""
import csv
import glob
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def per_dispatch(run_dir: str, counter: str) -> dict[str, list[float]]:
    files = glob.glob(os.path.join(run_dir, "**", "*counter_collection.csv"), recursive=True)
    out: dict[str, dict[str, float]] = {}
    for f in files:
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            k = r["Kernel_Name"]
            name = "k_env" if "k_env" in k else ("k_traffic" if "k_traffic" in k else None)
            if name is None:
                continue
            out.setdefault(name, {})
            out[name][r["Dispatch_Id"]] = out[name].get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
    return {k: [v[d] for d in sorted(v, key=int)] for k, v in out.items()}


def main():
    wl, fdir, wdir = sys.argv[1:4]
    tag = sys.argv[4] if len(sys.argv) > 4 else ""
    fetch, write = per_dispatch(fdir, "FETCH_SIZE"), per_dispatch(wdir, "WRITE_SIZE")
    sys.path.insert(0, ROOT)
    from bench import WORKLOADS
    envs = int(os.environ.get("PGTG_PMC_ENVS", "0")) or WORKLOADS[wl][2]
    rec = {"workload": wl, "envs": envs, "tag": tag, "unit": "bytes per step launch",
           "method": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE in separate bench.py runs; "
                     "read bytes = 2 x FETCH_SIZE (gfx950 16-B/lane streaming-read calibration), "
                     "write bytes = WRITE_SIZE; median over the step dispatches after the first 10 (tools/gpu_profile.sh: 200 warm-up + 60 steps)"}
    total = 0.0
    for k in ("k_env", "k_traffic"):
        if k not in fetch or k not in write:
            continue
        f = fetch[k][10:] or fetch[k]
        w = write[k][10:] or write[k]
        rb, wb = 2 * 1024 * statistics.median(f), 1024 * statistics.median(w)
        rec[k] = {"read_bytes": rb, "write_bytes": wb, "dispatches": [len(fetch[k]), len(write[k])]}
        total += rb + wb
    rec["hbm_bytes_per_launch"] = total
    p = os.path.join(ROOT, "profiles", f"pmc_{wl}.json")
    json.dump(rec, open(p, "w"), indent=1)
    print(json.dumps(rec))


if __name__ == "__main__":
    main()

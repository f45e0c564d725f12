"""SQ instruction counters of one workload's step kernels as the JSON bench.py reads for its issue
roofline (profiles/sq_<workload>.json).  Input: the two rocprofv3 --pmc passes of tools/sq_passes.sh.
Per kernel: the median over its dispatches of every counter summed over the device (wave-level
instruction counts: one per instruction a wave issues, whatever its active lanes).

Usage: python tools/sq_json.py <workload> <envs> <p1 dir> <p2 dir> > profiles/sq_<workload>.json"""
import csv
import glob
import json
import os
import statistics
import sys


def main():
    workload, envs, dirs = sys.argv[1], int(sys.argv[2]), sys.argv[3:]
    per: dict[str, dict[str, dict[int, float]]] = {}
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                k = r["Kernel_Name"]
                if "k_env" not in k and "k_traffic" not in k:
                    continue
                k = k.split("(")[0].replace("void ", "")
                c = per.setdefault(k, {}).setdefault(r["Counter_Name"], {})
                disp = int(r["Dispatch_Id"])
                c[disp] = c.get(disp, 0.0) + float(r["Counter_Value"])
    out = {"workload": workload, "envs": envs, "source": "rocprofv3 --pmc (tools/sq_passes.sh), median over dispatches",
           "kernels": {}}
    for k, cs in sorted(per.items()):
        out["kernels"][k] = {c: statistics.median(v.values()) for c, v in sorted(cs.items())}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()

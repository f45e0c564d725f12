#!/usr/bin/env python3
"""FETCH_SIZE / WRITE_SIZE calibration of the access widths the step kernels use (tools/micro/pmc_calib):
per kernel, the counter's bytes per dispatch (KB x 1024, median of 5) / the true 1 GiB.
Usage: python tools/pmc_calib.py <fetch_run_dir> <write_run_dir>  -> profiles/pmc_calibration.json"""
import csv
import glob
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def per_kernel(d, counter):
    out = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            k = r["Kernel_Name"].split("(")[0]
            out.setdefault(k, {}).setdefault(r["Dispatch_Id"], 0.0)
            out[k][r["Dispatch_Id"]] += float(r["Counter_Value"])
    return {k: statistics.median(v.values()) * 1024 for k, v in out.items()}


def main():
    fetch, write = per_kernel(sys.argv[1], "FETCH_SIZE"), per_kernel(sys.argv[2], "WRITE_SIZE")
    true = float(1 << 30)
    rec = {"true_bytes": true, "method": "tools/micro/pmc_calib.hip under rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE "
                                         "(separate runs); ratio = counter bytes / true bytes",
           "read": {k: {"fetch_bytes": v, "ratio": v / true} for k, v in fetch.items() if "k_read" in k},
           "write": {k: {"write_bytes": v, "ratio": v / true} for k, v in write.items() if "k_write" in k}}
    json.dump(rec, open(os.path.join(ROOT, "profiles", "pmc_calibration.json"), "w"), indent=1)
    print(json.dumps(rec))


if __name__ == "__main__":
    main()

"""Diagnostic: per-dispatch SQ counters of one kernel from rocprofv3 --pmc runs.

Usage: python tools/sq.py <kernel substring> <run_dir> [run_dir ...]
Prints, per dispatch of the matching kernel (in order), every counter summed over the device and,
when SQ_WAVES is present, divided by the wave count."""
import csv
import glob
import os
import sys


def main():
    kname, dirs = sys.argv[1], sys.argv[2:]
    rows: dict[tuple[int, str], float] = {}
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                if kname not in r["Kernel_Name"]:
                    continue
                key = (int(r["Dispatch_Id"]), r["Counter_Name"])
                rows[key] = rows.get(key, 0.0) + float(r["Counter_Value"])
    # dispatch ids differ between runs: index dispatches per counter in order
    by_counter: dict[str, list[float]] = {}
    for (disp, cname) in sorted(rows):
        by_counter.setdefault(cname, []).append(rows[(disp, cname)])
    waves = by_counter.get("SQ_WAVES")
    n = max(len(v) for v in by_counter.values())
    for i in range(n):
        parts = []
        for cname, vals in sorted(by_counter.items()):
            if i < len(vals):
                v = vals[i]
                per = f" ({v / waves[i]:.0f}/wave)" if waves and i < len(waves) and cname != "SQ_WAVES" else ""
                parts.append(f"{cname}={v:.0f}{per}")
        print(f"dispatch {i}: " + "  ".join(parts))


if __name__ == "__main__":
    main()

"""Diagnostic: issue/stall ratios of a kernel from the two SQ passes of tools/sq_passes.sh (median
over its dispatches).  Usage: python tools/sq_summary.py <kernel substring> <p1 dir> <p2 dir>"""
import csv
import glob
import os
import statistics
import sys


def main():
    kname, dirs = sys.argv[1], sys.argv[2:]
    per: dict[str, dict[int, float]] = {}
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                if kname not in r["Kernel_Name"]:
                    continue
                c = per.setdefault(r["Counter_Name"], {})
                disp = int(r["Dispatch_Id"])
                c[disp] = c.get(disp, 0.0) + float(r["Counter_Value"])
    med = {k: statistics.median(v.values()) for k, v in per.items()}
    w = med["SQ_WAVES"]
    cyc = med["SQ_WAVE_CYCLES"]
    out = {"kernel": kname, "waves": int(w), "wave_cycles": round(cyc / w),
           "valu_insts_per_wave": round(med["SQ_INSTS_VALU"] / w), "salu_insts_per_wave": round(med["SQ_INSTS_SALU"] / w),
           "lds_insts_per_wave": round(med["SQ_INSTS_LDS"] / w),
           "vmem_rd_per_wave": round(med["SQ_INSTS_VMEM_RD"] / w), "vmem_wr_per_wave": round(med["SQ_INSTS_VMEM_WR"] / w),
           "frac_waiting (WAIT_ANY/WAVE_CYCLES)": round(med["SQ_WAIT_ANY"] / cyc, 3),
           "frac_issuing_any (ACTIVE_INST_ANY/WAVE_CYCLES)": round(med["SQ_ACTIVE_INST_ANY"] / cyc, 3),
           "frac_valu (ACTIVE_INST_VALU/WAVE_CYCLES)": round(med["SQ_ACTIVE_INST_VALU"] / cyc, 3),
           "lds_bank_conflict_per_lds_inst": round(med["SQ_LDS_BANK_CONFLICT"] / max(1.0, med["SQ_INSTS_LDS"]), 2)}
    print(out)


if __name__ == "__main__":
    main()

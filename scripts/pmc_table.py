"""One row per rocprofv3 --pmc run directory (pmcN/) of the conv lab: the kernel the run profiled
(the longest-running dispatch name), its counters averaged over dispatches, and the derived ratios
MFMA-busy / (4 x CU-busy) (the MFMA counter sums the CU's 4 SIMDs), LDS-bank-conflict / LDS-active and LDS-wait / wave cycles.

usage: python scripts/pmc_table.py <dir with pmcN/ subdirs> [labels...]
"""
import collections
import csv
import glob
import os
import re
import sys


def digest(d):
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                name = row["Kernel_Name"]
                if "fill_bf16" in name:
                    continue
                vals[name][row["Counter_Name"]].append(float(row["Counter_Value"]))
    if not vals:
        return None, {}
    name = max(vals, key=lambda n: sum(vals[n].get("SQ_WAVE_CYCLES", [0])))
    return name, {k: sum(v) / len(v) for k, v in vals[name].items()}


def short(name):
    return re.sub(r"^void dlmpi::|\(dlmpi::\w+\)$", "", name).replace("unsigned short", "bf16")


def main():
    root = sys.argv[1]
    labels = sys.argv[2:]
    dirs = sorted(glob.glob(os.path.join(root, "pmc*/")), key=lambda p: int(re.sub(r"\D", "", os.path.basename(p[:-1])) or 0))
    print("| run | kernel | MFMA busy / CU busy | LDS bank conflict / LDS active | LDS wait / wave cycles |")
    print("|---|---|---:|---:|---:|")
    for i, d in enumerate(dirs):
        name, c = digest(d)
        if name is None:
            continue
        def r(a, b, k=1.0):
            return f"{c[a] / (k * c[b]):.3f}" if c.get(b) else "-"

        lab = labels[i] if i < len(labels) else os.path.basename(d[:-1])
        print(f"| {lab} | `{short(name)}` | {r('SQ_VALU_MFMA_BUSY_CYCLES', 'SQ_BUSY_CU_CYCLES', 4.0)} | "
              f"{r('SQ_LDS_BANK_CONFLICT', 'SQ_ACTIVE_INST_LDS')} | {r('SQ_WAIT_INST_LDS', 'SQ_WAVE_CYCLES')} |")


if __name__ == "__main__":
    main()

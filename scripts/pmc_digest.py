"""Digest rocprofv3 --pmc CSV runs (one counter group per run) of ONE kernel into a table.

usage: python scripts/pmc_digest.py <dir-with-pmcN/ subdirs> [--kernel SUBSTR] [--runs 1-4]

Every ``pmcN/**/c_counter_collection.csv`` is read; for each counter the value of the dispatches
whose name contains SUBSTR (default ``conv_igemm_kernel``) is averaged over dispatches (the warm-up
call included -- conv_one.py runs the same launch every iteration).  Derived ratios are printed
when their inputs were collected: MFMA-busy / CU-busy, VALU and LDS instructions per wave, bytes
fetched / written per dispatch.
"""
import argparse
import collections
import csv
import glob
import os


def read_run(d, sub):
    vals = collections.defaultdict(list)
    dur = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if sub not in row["Kernel_Name"]:
                    continue
                vals[row["Counter_Name"]].append(float(row["Counter_Value"]))
                dur.append(int(row["End_Timestamp"]) - int(row["Start_Timestamp"]))
    return {k: sum(v) / len(v) for k, v in vals.items()}, (sum(dur) / len(dur) if dur else 0.0)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("root")
    ap.add_argument("--kernel", default="conv_igemm_kernel")
    ap.add_argument("--runs", default=None, help="a-b: only pmc<a>..pmc<b>")
    a = ap.parse_args()
    runs = sorted(glob.glob(os.path.join(a.root, "pmc*")), key=lambda p: int("".join(c for c in os.path.basename(p) if c.isdigit()) or 0))
    runs = [r for r in runs if os.path.isdir(r)]
    if a.runs:
        lo, hi = map(int, a.runs.split("-"))
        runs = [r for r in runs if lo <= int("".join(c for c in os.path.basename(r) if c.isdigit())) <= hi]
    c = {}
    for r in runs:
        v, _ = read_run(r, a.kernel)
        c.update(v)
    for k in sorted(c):
        print(f"{k:32s} {c[k]:16.1f}")
    waves = c.get("SQ_WAVES")
    if "SQ_VALU_MFMA_BUSY_CYCLES" in c and "SQ_BUSY_CU_CYCLES" in c:
        print(f"{'MFMA busy / CU busy / 4 SIMDs':32s} {c['SQ_VALU_MFMA_BUSY_CYCLES'] / max(1.0, c['SQ_BUSY_CU_CYCLES']) / 4:16.3f}")
    if waves:
        for k in ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_MFMA", "SQ_INSTS_SALU", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR"):
            if k in c:
                print(f"{k + ' / wave':32s} {c[k] / waves:16.1f}")
    if "SQ_WAIT_INST_ANY" in c and "SQ_WAVE_CYCLES" in c:
        print(f"{'wait-inst / wave-cycles':32s} {c['SQ_WAIT_INST_ANY'] / max(1.0, c['SQ_WAVE_CYCLES']):16.3f}")
    if "SQ_LDS_BANK_CONFLICT" in c and "SQ_ACTIVE_INST_LDS" in c:
        print(f"{'LDS conflict / LDS active':32s} {c['SQ_LDS_BANK_CONFLICT'] / max(1.0, c['SQ_ACTIVE_INST_LDS']):16.3f}")


if __name__ == "__main__":
    main()

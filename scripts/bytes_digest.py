"""Per-kernel HBM bytes of a bench.py run profiled by scripts/bytes.sh (rocprofv3 --pmc FETCH_SIZE /
WRITE_SIZE, one pass each): per-step fetch / write GB, the isolated duration and the resulting GB/s per
kernel name, sorted by bytes.

usage: python scripts/bytes_digest.py <fetch dir> <write dir> [--steps N]   (N = steps in the trace)
"""
import argparse
import collections
import csv
import glob
import os


def read(d, ctr):
    val = collections.defaultdict(float)
    dur = collections.defaultdict(float)
    cnt = collections.Counter()
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row["Counter_Name"] != ctr:
                    continue
                name = row["Kernel_Name"].split("(")[0].replace("void ", "")[:70]
                val[name] += float(row["Counter_Value"]) * 1024.0   # KB -> bytes
                dur[name] += (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) * 1e-9
                cnt[name] += 1
    return val, dur, cnt


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch")
    ap.add_argument("write")
    ap.add_argument("--steps", type=float, default=1.0)
    a = ap.parse_args()
    fv, fd, fc = read(a.fetch, "FETCH_SIZE")
    wv, wd, wc = read(a.write, "WRITE_SIZE")
    names = set(fv) | set(wv)
    rows = []
    for n in names:
        f, w = fv.get(n, 0.0) / a.steps, wv.get(n, 0.0) / a.steps
        d = (fd.get(n, 0.0) + wd.get(n, 0.0)) / 2 / a.steps
        rows.append((f + w, n, f, w, d, fc.get(n, 0) / a.steps))
    rows.sort(reverse=True)
    tf = sum(r[2] for r in rows)
    tw = sum(r[3] for r in rows)
    td = sum(r[4] for r in rows)
    print(f"per step: fetch {tf / 1e9:.2f} GB, write {tw / 1e9:.2f} GB, serialized kernel time {td * 1e3:.2f} ms\n")
    print("| kernel | calls | fetch GB | write GB | ms (serialized) | TB/s |")
    print("|---|---:|---:|---:|---:|---:|")
    for tot, n, f, w, d, c in rows[:40]:
        print(f"| `{n}` | {c:.0f} | {f / 1e9:.3f} | {w / 1e9:.3f} | {d * 1e3:.3f} | {tot / d / 1e12 if d else 0:.2f} |")


if __name__ == "__main__":
    main()

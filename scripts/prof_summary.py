"""Digest rocprofv3 kernel statistics into a per-step markdown table.

usage: python scripts/prof_summary.py <kernel_stats.csv | results.db> [--steps N] [--top K] [--skip-first M]

Input: a ``*_kernel_stats.csv`` (``--output-format csv``) or the rocpd SQLite database rocprofv3
writes by default (``*_results.db``, its ``kernels`` view).  ``--steps`` = number of profiled
training steps to normalise to ms/step.  With a database, ``--skip-first M`` drops the dispatches of
the first M seconds of GPU time is not possible to know, so ``--window LAST_SECONDS`` keeps only the
dispatches that start in the last LAST_SECONDS of the trace (e.g. the timed steps after warm-up).
"""
import argparse
import csv
import re
import sqlite3


def short(name: str) -> str:
    name = re.sub(r"\(.*", "", name) if "<" not in name else name
    name = name.replace("void ", "").replace("dlmpi::", "")
    return name[:90]


def rows_from_db(path, window_s=None):
    c = sqlite3.connect(path)
    q = "select name, start, end from kernels"
    ks = c.execute(q).fetchall()
    if window_s:
        tend = max(k[2] for k in ks)
        ks = [k for k in ks if k[1] >= tend - window_s * 1e9]
    agg = {}
    for name, s, e in ks:
        a = agg.setdefault(name, [0, 0.0])
        a[0] += 1
        a[1] += e - s
    return [{"Name": n, "Calls": v[0], "TotalDurationNs": v[1]} for n, v in agg.items()]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--steps", type=float, default=1.0)
    ap.add_argument("--top", type=int, default=25)
    ap.add_argument("--window", type=float, default=None, help="(db) keep dispatches of the last N seconds")
    ap.add_argument("--step-kernel", default=None,
                    help="count training steps as the calls of this once-per-step kernel (overrides --steps)")
    a = ap.parse_args()
    if a.path.endswith(".db"):
        rows = rows_from_db(a.path, a.window)
    else:
        rows = list(csv.DictReader(open(a.path)))
    if a.step_kernel:
        a.steps = float(sum(int(r["Calls"]) for r in rows if short(r["Name"]).startswith(a.step_kernel)))
        print(f"steps in window: {a.steps:.0f} (calls of {a.step_kernel})\n")
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    print("| kernel | calls/step | ms/step | % |\n|---|---:|---:|---:|")
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:a.top]:
        t = float(r["TotalDurationNs"])
        print(f"| `{short(r['Name'])}` | {int(r['Calls']) / a.steps:.0f} | {t / 1e6 / a.steps:.3f} | "
              f"{100 * t / tot:.1f} |")
    print(f"| **total** | | **{tot / 1e6 / a.steps:.3f}** | 100 |")


if __name__ == "__main__":
    main()

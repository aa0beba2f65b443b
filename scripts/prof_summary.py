"""Digest a rocprofv3 ``*_kernel_stats.csv`` into a per-step markdown table.

usage: python scripts/prof_summary.py <kernel_stats.csv> [--steps N] [--top K]
``--steps`` = number of profiled training steps (incl. warmup) to normalise to ms/step.
"""
import argparse
import csv
import re


def short(name: str) -> str:
    name = re.sub(r"\(.*", "", name) if "<" not in name else name
    name = name.replace("void ", "").replace("dlmpi::", "")
    return name[:90]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--steps", type=float, default=1.0)
    ap.add_argument("--top", type=int, default=25)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.csv)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    print(f"| kernel | calls/step | ms/step | % |\n|---|---:|---:|---:|")
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:a.top]:
        t = float(r["TotalDurationNs"])
        print(f"| `{short(r['Name'])}` | {int(r['Calls']) / a.steps:.0f} | {t / 1e6 / a.steps:.3f} | "
              f"{100 * t / tot:.1f} |")
    print(f"| **total** | | **{tot / 1e6 / a.steps:.3f}** | 100 |")


if __name__ == "__main__":
    main()

"""Per-kernel-family ms/step of two rocpd databases (the last complete step of each), side by side.
usage: python scripts/prof_compare.py a_results.db b_results.db"""
import collections
import re
import sqlite3
import sys


def step_kernels(path):
    c = sqlite3.connect(path)
    ks = c.execute("select name, start, end, stream_id from kernels order by start").fetchall()
    idx = [i for i, k in enumerate(ks) if "sgd_kernel" in k[0] or "adam_kernel" in k[0]]
    return ks[idx[-2] + 1: idx[-1] + 1]


def family(name):
    n = name.replace("void ", "").replace("dlmpi::", "")
    n = re.sub(r"\(.*", "", n)
    return n[:60]


def main():
    res = []
    for p in sys.argv[1:3]:
        agg = collections.defaultdict(lambda: [0, 0.0])
        ks = step_kernels(p)
        for name, s, e, st in ks:
            a = agg[(family(name), st)]
            a[0] += 1
            a[1] += (e - s) / 1e3
        res.append((agg, (ks[-1][2] - ks[0][1]) / 1e3))
    keys = sorted(set(res[0][0]) | set(res[1][0]), key=lambda k: -max(res[0][0].get(k, [0, 0])[1], res[1][0].get(k, [0, 0])[1]))
    print(f"{'kernel':60s} {'str':>3s} | {'A n':>4s} {'A us':>8s} | {'B n':>4s} {'B us':>8s} | {'A-B us':>8s}")
    for k in keys[:40]:
        a, b = res[0][0].get(k, [0, 0.0]), res[1][0].get(k, [0, 0.0])
        print(f"{k[0]:60s} {k[1]:3d} | {a[0]:4d} {a[1]:8.0f} | {b[0]:4d} {b[1]:8.0f} | {a[1] - b[1]:8.0f}")
    for s in sorted({k[1] for k in keys}):
        ta = sum(v[1] for k, v in res[0][0].items() if k[1] == s)
        tb = sum(v[1] for k, v in res[1][0].items() if k[1] == s)
        print(f"stream {s}: A {ta:.0f} us  B {tb:.0f} us")
    print(f"step span: A {res[0][1]:.0f} us  B {res[1][1]:.0f} us")


if __name__ == "__main__":
    main()

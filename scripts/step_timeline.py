"""Print one steady-state step of a rocprofv3 kernel trace as a timeline (start, duration, stream,
grid, kernel), between the last two optimizer kernels.

usage: python scripts/step_timeline.py <results.db> [--marker sgd_kernel] [--stream N]
"""
import argparse
import re
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--marker", default="sgd_kernel")
    ap.add_argument("--stream", type=int, default=None)
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    ks = c.execute("select name, start, end, stream_id, grid_x, grid_y, grid_z from kernels order by start").fetchall()
    mk = [i for i, k in enumerate(ks) if a.marker in k[0]]
    step = ks[mk[-2] + 1:mk[-1] + 1]
    t0 = step[0][1]
    for k in step:
        if a.stream is not None and k[3] != a.stream:
            continue
        n = re.sub(r"\(.*", "", k[0]).replace("void ", "").replace("dlmpi::", "")[:70]
        print(f"{(k[1] - t0) / 1e3:8.1f} {(k[2] - k[1]) / 1e3:7.1f} s{k[3]} {k[4]:>8} {k[5]} {k[6]} {n}")


if __name__ == "__main__":
    main()

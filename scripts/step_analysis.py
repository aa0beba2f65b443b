"""One steady-state training step from a rocprofv3 kernel-trace database (rocpd ``*_results.db``).

usage: python scripts/step_analysis.py <results.db> [--marker sgd_kernel|adam_kernel] [--step -2] [--top 15]

The step is the dispatch range between two consecutive optimizer kernels (``--marker``; ``--step``
picks which pair, default the second-to-last).  Printed: span, per-stream busy time, GPU busy
(union of all streams), time with exactly one kernel in flight and idle gaps, the kernels that run
ALONE the longest (the serial critical path), and the idle gaps of stream 0 (the main stream)
grouped by the kernel that follows them.
"""
import argparse
import collections
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--marker", default="sgd_kernel")
    ap.add_argument("--step", type=int, default=-2)
    ap.add_argument("--top", type=int, default=15)
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = c.execute("select name, start, end, stream_id from kernels order by start").fetchall()
    marks = [i for i, r in enumerate(rows) if a.marker in r[0]]
    if len(marks) < 2:
        raise SystemExit(f"fewer than two '{a.marker}' dispatches")
    i0, i1 = marks[a.step - 1], marks[a.step]
    seg = rows[i0 + 1:i1 + 1]
    t0 = seg[0][1]
    span = (seg[-1][2] - t0) / 1e3
    busy = collections.defaultdict(float)
    for _, s, e, st in seg:
        busy[st] += (e - s) / 1e3
    ev = sorted([(s, 1, i) for i, (_, s, e, _) in enumerate(seg)] + [(e, -1, i) for i, (_, s, e, _) in enumerate(seg)])
    act, last = set(), None
    one = zero = 0.0
    alone = collections.defaultdict(float)
    for t, d, i in ev:
        if last is not None:
            if len(act) == 1:
                one += t - last
                alone[seg[next(iter(act))][0][:70]] += t - last
            elif not act:
                zero += t - last
        if d == 1:
            act.add(i)
        else:
            act.discard(i)
        last = t
    print(f"dispatches {len(seg)}  span {span:.1f} us")
    print("per-stream busy (us):", {k: round(v, 1) for k, v in sorted(busy.items())})
    print(f"GPU busy {span - zero / 1e3:.1f} us; exactly one kernel in flight {one / 1e3:.1f} us; idle {zero / 1e3:.1f} us")
    print("\nlongest ALONE (us):")
    for k, v in sorted(alone.items(), key=lambda x: -x[1])[:a.top]:
        print(f"{v / 1e3:9.1f}  {k}")
    main = sorted((s, e, n) for n, s, e, st in seg if st == seg[0][3])
    gaps = collections.defaultdict(lambda: [0, 0.0])
    for (s0, e0, _), (s1, e1, n1) in zip(main, main[1:]):
        g = s1 - max(e0, s0)
        if g > 0:
            gaps[n1[:70]][0] += 1
            gaps[n1[:70]][1] += g / 1e3
    tot = sum(v[1] for v in gaps.values())
    print(f"\nstream {seg[0][3]} idle gaps: {tot:.1f} us total; by the kernel that follows (count, us):")
    for k, v in sorted(gaps.items(), key=lambda x: -x[1][1])[:a.top]:
        print(f"{v[0]:5d} {v[1]:9.1f}  {k}")


if __name__ == "__main__":
    main()

"""Attribute the D2D copy kernels (__amd_rocclr_copyBuffer) and ATen kernels of a traced bench step
to the HIP API calls that issued them and the kernels launched around them (scripts/copytrace.sh).

usage: python scripts/copytrace.py <rocprofv3 output dir>
"""
import collections
import csv
import glob
import os
import sys


def rows(d, pat):
    out = []
    for f in glob.glob(os.path.join(d, "**", pat), recursive=True):
        with open(f) as fh:
            out += list(csv.DictReader(fh))
    return out


def main():
    d = sys.argv[1]
    api = rows(d, "*hip_api_trace.csv")
    ker = rows(d, "*kernel_trace.csv")
    api.sort(key=lambda r: int(r["Start_Timestamp"]))
    # the API calls in issue order; kernel launches (hipLaunchKernel / hipModuleLaunchKernel / ExtLaunch)
    # carry the correlation id of their kernel
    kname = {r["Correlation_Id"]: r["Kernel_Name"] for r in ker}
    seq = []
    for r in api:
        fn = r["Function"]
        cid = r["Correlation_Id"]
        name = kname.get(cid)
        seq.append((fn, name))
    # only the timed steps: between bench.py's two clock-stamp launches
    marks = [i for i, (_, n) in enumerate(seq) if n and "clock_stamp" in n]
    if len(marks) >= 2:
        seq = seq[marks[0] + 1:marks[-1]]
        print(f"timed region: {len(seq)} API calls, "
              f"{sum(1 for f, n in seq if n)} kernels, {sum(1 for f, n in seq if f.startswith('hipMemcpy'))} memcpy calls")
    ctx = collections.Counter()
    for i, (fn, name) in enumerate(seq):
        interesting = fn.startswith("hipMemcpy") or (name and ("copyBuffer" in name or "at::native" in name))
        if not interesting:
            continue
        prev = next((seq[j][1] for j in range(i - 1, max(-1, i - 40), -1) if seq[j][1] and "copyBuffer" not in seq[j][1]), None)
        nxt = next((seq[j][1] for j in range(i + 1, min(len(seq), i + 40)) if seq[j][1] and "copyBuffer" not in seq[j][1]), None)
        short = lambda s: (s or "-").split("(")[0].replace("void ", "")[:60]  # noqa: E731
        ctx[(fn, short(name), short(prev), short(nxt))] += 1
    print("count | API | kernel | previous kernel | next kernel")
    for (fn, name, prev, nxt), c in ctx.most_common(60):
        print(f"{c:5d} | {fn} | {name} | {prev} | {nxt}")


if __name__ == "__main__":
    main()

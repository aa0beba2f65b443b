"""Per-kernel register / spill / LDS audit of the gfx950 code objects (hipcc's resource-usage
remarks, the same numbers as `.vgpr_count` / `.vgpr_spill_count` / `.agpr_count` in the notes).

python scripts/regs.py [--spills-only] [FILE.hip ...]     (default: every csrc/kernels/*.hip)
Exit status 1 if any kernel spills."""
import argparse
import concurrent.futures as cf
import glob
import os
import re
import subprocess
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KDIR = os.path.join(HERE, "deeplearning_mpi_amd", "csrc", "kernels")
FIELDS = ("VGPRs", "AGPRs", "VGPRs Spill", "SGPRs Spill", "ScratchSize [bytes/lane]", "Occupancy [waves/SIMD]",
          "LDS Size [bytes/block]")


def audit(path):
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-munsafe-fp-atomics",
           "-Rpass-analysis=kernel-resource-usage", "--cuda-device-only", "-c", path, "-o", os.devnull]
    out = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True).stdout
    rows, cur = [], None
    for line in out.splitlines():
        m = re.search(r"remark:\s+(.*?)\s*\[-Rpass-analysis", line)
        if not m:
            continue
        txt = m.group(1)
        if txt.startswith("Function Name:"):
            cur = {"name": txt.split(":", 1)[1].strip(), "file": os.path.basename(path)}
            rows.append(cur)
        elif cur is not None and ":" in txt:
            k, v = txt.rsplit(":", 1)
            if k.strip() in FIELDS:
                cur[k.strip()] = v.strip()
    return rows


def demangle(names):
    try:
        out = subprocess.run(["c++filt"], input="\n".join(names), stdout=subprocess.PIPE, text=True).stdout
        return out.splitlines()
    except OSError:
        return names


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("files", nargs="*")
    ap.add_argument("--spills-only", action="store_true")
    a = ap.parse_args()
    files = a.files or sorted(glob.glob(os.path.join(KDIR, "*.hip")))
    with cf.ThreadPoolExecutor(max_workers=min(8, os.cpu_count() or 4)) as ex:
        rows = [r for rs in ex.map(audit, files) for r in rs]
    names = demangle([r["name"] for r in rows])
    spills = 0
    print(f"{'vgpr':>5} {'agpr':>5} {'vspl':>5} {'sspl':>5} {'scr':>4} {'occ':>3} {'lds':>6}  kernel")
    for r, n in zip(rows, names):
        sp = int(r.get("VGPRs Spill", 0)) + int(r.get("SGPRs Spill", 0))
        spills += sp > 0
        if a.spills_only and sp == 0:
            continue
        print(f"{r.get('VGPRs', '?'):>5} {r.get('AGPRs', '?'):>5} {r.get('VGPRs Spill', '?'):>5} {r.get('SGPRs Spill', '?'):>5} {r.get('ScratchSize [bytes/lane]', '?'):>4} "
              f"{r.get('Occupancy [waves/SIMD]', '?'):>3} {r.get('LDS Size [bytes/block]', '?'):>6}  {n[:110]}")
    print(f"{len(rows)} kernels, {spills} spilling")
    sys.exit(1 if spills else 0)


if __name__ == "__main__":
    main()

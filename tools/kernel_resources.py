#!/usr/bin/env python3
"""Per-kernel register / scratch / LDS use of every HIP translation unit (device assembly metadata).
Flags kernels that spill to scratch.  Run after editing a kernel:  python tools/kernel_resources.py
"""
import concurrent.futures as cf
import glob
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "crypto3-fil-proofs_amd", "csrc")


def one(src):
    out = f"/tmp/kres_{os.path.basename(src)}.s"
    subprocess.check_call(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-fno-gpu-rdc",
                           "--offload-device-only", "-w", "-S", src, "-o", out])
    s = open(out).read()
    rows = []
    for b in s.split("  - .agpr_count:")[1:]:
        name = re.search(r"\.name:\s+(\S+)", b).group(1)
        if not name.startswith("_ZN2mi"):
            continue
        g = lambda k: int((re.search(r"\." + k + r":\s+(\d+)", b) or [0, 0])[1])
        agpr = int(b.split("\n")[0].strip())
        rows.append((os.path.basename(src), name, g("vgpr_count"), agpr, g("vgpr_spill_count"),
                     g("private_segment_fixed_size"), g("group_segment_fixed_size")))
    return rows


def main():
    srcs = sorted(glob.glob(os.path.join(CSRC, "*.hip")))
    with cf.ThreadPoolExecutor(8) as ex:
        allrows = [r for rows in ex.map(one, srcs) for r in rows]
    bad = 0
    for tu, name, v, a, spill, scratch, lds in allrows:
        m = re.search(r"(k_\w+?)(I|E)", name)
        short = m.group(1) if m else name[:40]
        tag = "SPILL" if scratch else ""
        bad += bool(scratch)
        if scratch or v > 128 or "-a" in sys.argv:
            print(f"{tu:12s} {short:28s} vgpr={v:3d} agpr={a:3d} spill={spill:4d} scratch={scratch:5d} lds={lds:6d} {tag}")
    print(f"{len(allrows)} kernels, {bad} with scratch")


if __name__ == "__main__":
    main()

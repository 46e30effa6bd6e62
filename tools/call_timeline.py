#!/usr/bin/env python3
"""Per-stream view of one Winning-PoSt call from a rocprofv3 SQLite trace (kernel + HIP runtime traces):
each stream's first / last kernel and busy time, the call's kernel-free gaps, and the HIP calls that block a
host thread for more than --min-ms.

    python tools/call_timeline.py gpurun_out/win4/trace/run_results.db [--call -2] [--min-ms 0.3]
"""
import argparse
import collections
import os
import sqlite3
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from rocpd_summary import short  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--call", type=int, default=-2)
    ap.add_argument("--min-ms", type=float, default=0.3)
    ap.add_argument("--kernels", action="store_true", help="each stream's kernels (start, duration) in call order")
    a = ap.parse_args()
    db = sqlite3.connect(a.db)
    k = [(short(n), s, e, st) for n, s, e, st in db.execute("select name, start, end, stream_id from kernels order by start")]
    starts = [i for i in range(len(k)) if "k_wit" in k[i][0] and (i == 0 or "k_wit" not in k[i - 1][0])]
    lo = starts[a.call]
    hi = starts[a.call + 1] if a.call + 1 < 0 or a.call + 1 < len(starts) else len(k)
    sel = k[lo:hi]
    t0, t1 = sel[0][1], k[hi][1] if hi < len(k) else max(e for _, _, e, _ in sel)
    print(f"call: {(t1 - t0) / 1e6:.2f} ms from its first kernel to the next call's")
    per = collections.defaultdict(list)
    for n, s, e, st in sel:
        per[st].append((n, (s - t0) / 1e6, (e - t0) / 1e6))
    for st, v in per.items():
        print(f"stream {st}: {len(v)} kernels, {v[0][1]:.2f} .. {max(e for _, _, e in v):.2f} ms, busy {sum(e - s for _, s, e in v):.2f}")
        if a.kernels:  # runs of one kernel name merged
            run = None
            for n, s, e in v:
                if run and run[0] == n and s - run[2] < 0.05:
                    run = (n, run[1], e, run[3] + 1, run[4] + e - s)
                else:
                    if run:
                        print(f"    {run[1]:7.3f} +{run[2] - run[1]:6.3f} ms  x{run[3]:<3d} busy {run[4]:.3f}  {run[0]}")
                    run = (n, s, e, 1, e - s)
            if run:
                print(f"    {run[1]:7.3f} +{run[2] - run[1]:6.3f} ms  x{run[3]:<3d} busy {run[4]:.3f}  {run[0]}")
    iv = sorted((s, e) for _, s, e in sum(per.values(), []))
    gaps, cur = [], iv[0][1]
    for s, e in iv[1:]:
        if s > cur + 0.2:
            gaps.append((cur, s))
        cur = max(cur, e)
    print("kernel-free gaps > 0.2 ms:", ", ".join(f"{g0:.2f}-{g1:.2f}" for g0, g1 in gaps))
    try:
        regs = list(db.execute("select name, start, end, tid from regions where start >= ? and start < ? order by start", (t0, t1)))
    except sqlite3.Error:
        regs = []
    for n, s, e, tid in regs:
        if (e - s) / 1e6 >= a.min_ms:
            print(f"  host tid {tid}: {(s - t0) / 1e6:6.2f} + {(e - s) / 1e6:5.2f} ms {n}")


if __name__ == "__main__":
    main()

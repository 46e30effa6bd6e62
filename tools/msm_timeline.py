#!/usr/bin/env python3
"""Per-call timeline of standalone MSMs from a rocprofv3 --kernel-trace SQLite output (tools/msm_bench.py run
under the profiler).  A call starts at each digit kernel (k_digits*); the last `--reps` calls are summarised:
span (first kernel start to last kernel end), device-busy time, the kernel-free gaps (host round trips and launch
latency) and device time per kernel.

    python tools/msm_timeline.py gpurun_out/msm20/trace/run_results.db [--reps 10]
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
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    db = sqlite3.connect(a.db)
    rows = [(short(n), s, e) for n, s, e in db.execute("select name, start, end from kernels order by start")]
    firsts = [i for i, r in enumerate(rows) if r[0].startswith("k_digits")]
    calls = [(firsts[k], firsts[k + 1] if k + 1 < len(firsts) else len(rows)) for k in range(len(firsts))]
    calls = calls[-a.reps:]
    per = collections.OrderedDict()
    spans, busys, gaps = [], [], []
    nk = 0
    for lo, hi in calls:
        sel = rows[lo:hi]
        nk += len(sel)
        t0, t1 = sel[0][1], max(e for _, _, e in sel)
        spans.append((t1 - t0) / 1e6)
        b, ce = 0, None
        big = []
        for n, s, e in sorted(sel, key=lambda r: r[1]):
            if ce is not None and s > ce:
                if s - ce > 20000:
                    big.append(((s - ce) / 1e6, n))
                b += e - s if e > s else 0
            else:
                b += max(0, e - (ce if ce is not None else s))
            ce = e if ce is None else max(ce, e)
            per.setdefault(n, [0.0, 0])
            per[n][0] += (e - s) / 1e6
            per[n][1] += 1
        busys.append(b / 1e6)
        gaps.append(big)
    r = len(calls)
    print(f"{r} calls: span {sum(spans) / r:.3f} ms, busy {sum(busys) / r:.3f} ms, {nk / r:.0f} kernels per call")
    print("gaps > 20 us in the last call (ms, next kernel): " + ", ".join(f"{g:.3f} {n}" for g, n in gaps[-1]))
    print("| kernel | ms per call | launches per call |\n|---|---|---|")
    for n, (ms, cnt) in sorted(per.items(), key=lambda kv: -kv[1][0]):
        print(f"| {n} | {ms / r:.3f} | {cnt / r:.1f} |")


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Device-time breakdown of the Winning-PoSt latency leg from a rocprofv3 --kernel-trace SQLite output
(tools/winning_prof.sh: bench.py with only that leg after a tiny main leg).

A Winning-PoSt call = the GPU witness (k_wit_* kernels) then the proof.  Calls are found as the runs of kernels
that start with a witness kernel after a non-witness kernel; the last `--reps` calls are summarised: wall span
per call (first kernel start to last kernel end), the union of kernel intervals over every stream (busy) and
the idle rest, and device time per kernel class.

    python tools/winning_timeline.py gpurun_out/win/trace/run_results.db [--reps 10] [--md]
"""
import argparse
import collections
import os
import sqlite3
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from lane_timeline import klass  # noqa: E402
from rocpd_summary import short  # noqa: E402


def union_ms(iv):
    tot, cur_s, cur_e = 0, None, None
    for s, e in sorted(iv):
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot / 1e6


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--md", action="store_true")
    ap.add_argument("--top", type=int, default=0, help="also list the N kernels with the most device time per call")
    a = ap.parse_args()
    db = sqlite3.connect(a.db)
    rows = [(short(n), s, e) for n, s, e in db.execute("select name, start, end from kernels order by start")]
    starts = [i for i in range(len(rows)) if rows[i][0].startswith("stacked::") or "k_wit" in rows[i][0]]
    first = [i for i in starts if i == 0 or not ("k_wit" in rows[i - 1][0])]
    calls = [(first[k], first[k + 1] if k + 1 < len(first) else len(rows)) for k in range(len(first))]
    calls = calls[-a.reps:]
    spans, busy = [], []
    cls = collections.OrderedDict()
    per_kernel = collections.defaultdict(lambda: [0, 0.0])
    wit = []
    for lo, hi in calls:
        sel = rows[lo:hi]
        t0, t1 = sel[0][1], max(e for _, _, e in sel)
        spans.append((t1 - t0) / 1e6)
        busy.append(union_ms([(s, e) for _, s, e in sel]))
        w = [(s, e) for n, s, e in sel if "k_wit" in n]
        wit.append(union_ms(w))
        for n, s, e in sel:
            k = "witness (k_wit_*)" if "k_wit" in n else klass(n)
            cls[k] = cls.get(k, 0.0) + (e - s) / 1e6
            per_kernel[n][0] += 1
            per_kernel[n][1] += (e - s) / 1e6
    n = len(calls)
    out = {"calls": n, "span_ms_mean": sum(spans) / n, "busy_ms_mean": sum(busy) / n,
           "idle_ms_mean": (sum(spans) - sum(busy)) / n, "witness_busy_ms_mean": sum(wit) / n,
           "kernels_per_call": sum(hi - lo for lo, hi in calls) / n,
           "class_ms_per_call": {k: round(v / n, 3) for k, v in cls.items()}}
    if a.md:
        print(f"Winning-PoSt call: span {out['span_ms_mean']:.2f} ms, kernels busy {out['busy_ms_mean']:.2f} ms, "
              f"idle {out['idle_ms_mean']:.2f} ms, {out['kernels_per_call']:.0f} kernels per call\n")
        print("| class | device ms per call (sum over streams) |\n|---|---|")
        for k, v in out["class_ms_per_call"].items():
            print(f"| {k} | {v:.3f} |")
        if a.top:
            print("\n| kernel | launches per call | device ms per call |\n|---|---|---|")
            for name, (cnt, ms) in sorted(per_kernel.items(), key=lambda kv: -kv[1][1])[:a.top]:
                print(f"| `{name[:70]}` | {cnt / n:g} | {ms / n:.2f} |")
    else:
        import json

        print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Per-stream timeline and per-class device time of ONE timed proof from a rocprofv3 --kernel-trace SQLite
output (tools/lane_prof.sh / tools/lane_prof1.sh).

The proof window runs from the second-to-last k_copy_to_mont (start of a proof's witness map on the main
lane) to the last one, so with `bench.py --steps 3 --warmup 1` it is the second timed proof, with the next
proof's upload and the previous one's tail around it.  Consecutive launches of one kernel are merged into
one timeline row.

    python tools/lane_timeline.py gpurun_out/lane0/trace/run_results.db [--rows] [--md]
"""
import argparse
import collections
import os
import sqlite3
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from rocpd_summary import short  # noqa: E402

CLASSES = [
    ("G1 accumulation (H, L, A, B_G1)", ("k_accum_level0<Fq>",)),
    ("G2 accumulation (B_G2 + second level)", ("k_accum_level0<Fq2>",)),
    ("bucket reduction (G1 + G2)", ("k_bucket_reduce", "k_seg_fold", "k_sum_groups", "k_tree_level",
                                    "k_bucket_affine", "k_glv_merge")),
    ("NTT (7 transforms) + QAP division", ("k_ntt_pass", "k_qap_divide", "k_ntt_")),
    ("digits + sort + bounds", ("k_digits", "radix_sort", "k_bounds", "k_l2_digits", "k_chunk", "k_end_to_cnt",
                                "k_flag_multi", "k_tree_count", "k_tree_heads", "merge_sort", "scan",
                                "init_lookback", "partition", "reduce_config", "transform")),
    ("fills / copies", ("__amd_rocclr",)),
    ("witness map", ("k_eval_rows", "k_eval_blocks", "k_eval_tail", "k_copy_to_mont")),
]


def klass(name):
    for cname, keys in CLASSES:
        if any(k in name for k in keys):
            return cname
    return "rest"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--rows", action="store_true", help="print the merged per-stream timeline")
    ap.add_argument("--min-ms", type=float, default=0.5)
    a = ap.parse_args()
    db = sqlite3.connect(a.db)
    rows = list(db.execute("select name, start, end, stream_id from kernels order by start"))
    marks = [r[1] for r in rows if "k_copy_to_mont" in r[0]]
    if len(marks) < 2:
        sys.exit("need at least two proofs in the trace")
    t0, t1 = marks[-2], marks[-1]
    sel = [(short(n), s, e, st) for n, s, e, st in rows if t0 <= s < t1]
    acc = collections.OrderedDict((c, 0.0) for c, _ in CLASSES)
    acc["rest"] = 0.0
    for n, s, e, _ in sel:
        acc[klass(n)] += (e - s) / 1e6
    by = collections.defaultdict(list)
    for r in sel:
        by[r[3]].append(r)
    print(f"proof window {(t1 - t0) / 1e6:.1f} ms")
    # union of the kernels' busy intervals over all streams: the window minus this is time with no kernel
    # running at all (host synchronisations, launch gaps)
    union, cur_s, cur_e = 0, None, None
    for _, s, e, _ in sorted(sel, key=lambda r: r[1]):
        e = min(e, t1)
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                union += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        union += cur_e - cur_s
    print(f"device busy (union over streams) {union / 1e6:.1f} ms, idle {(t1 - t0 - union) / 1e6:.1f} ms")
    for st, rs in sorted(by.items()):
        busy = sum(e - s for _, s, e, _ in rs) / 1e6
        print(f"stream {st}: {len(rs)} launches, busy {busy:.1f} ms, span {(rs[-1][2] - rs[0][1]) / 1e6:.1f} ms")
        if a.rows:
            cur, first, tot, cnt = None, 0, 0, 0
            merged = []
            for n, s, e, _ in rs:
                if n != cur:
                    if cur:
                        merged.append((cur, first, tot, cnt))
                    cur, first, tot, cnt = n, s, 0, 0
                tot += e - s
                cnt += 1
            merged.append((cur, first, tot, cnt))
            for n, s, tot, cnt in merged:
                if tot / 1e6 >= a.min_ms:
                    print(f"  {(s - t0) / 1e6:8.1f} {tot / 1e6:8.2f} ms x{cnt:<4d} {n}")
    print("| class | device ms |\n|---|---|")
    for k, v in acc.items():
        print(f"| {k} | {v:.1f} |")
    print(f"| **sum of kernel time** | **{sum(acc.values()):.1f}** |")
    print(f"| **proof window** | **{(t1 - t0) / 1e6:.1f}** |")
    per = collections.defaultdict(float)
    for n, s, e, _ in sel:
        per[n] += (e - s) / 1e6
    print("top kernels:")
    for n, v in sorted(per.items(), key=lambda kv: -kv[1])[:20]:
        print(f"  {v:8.2f} ms  {n}")


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Kernel statistics from a rocprofv3 SQLite output (``run_results.db``), for runs made without
``--output-format csv``.  Writes the same columns as rocprofv3's kernel_stats.csv.

    python tools/rocpd_summary.py gpurun_out/p2/trace/run_results.db [--csv out.csv] [--timeline]
"""
import argparse
import csv
import re
import sqlite3
import sys


def short(name):
    name = name.replace("(anonymous namespace)::", "").replace("void ", "")
    name = re.sub(r"ROCPRIM_\d+_NS::", "", name)
    m = re.match(r"rocprim::detail::trampoline_kernel<rocprim::detail::(\w+)", name)
    if m:
        return "rocprim::" + m.group(1)
    m = re.match(r"rocprim::(?:detail::)?(\w+)", name)
    if m:
        return "rocprim::" + m.group(1)
    name = re.sub(r"\(.*$", "", name)
    name = re.sub(r"^mi::", "", name)
    name = re.sub(r"mi::Fp<mi::FqDesc>|mi::fq_t", "Fq", name)
    name = re.sub(r"mi::fq2_t", "Fq2", name)
    return name[:90]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--csv")
    ap.add_argument("--timeline", action="store_true")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = list(c.execute("select name, start, end from kernels order by start"))
    agg = {}
    for name, s, e in rows:
        k = short(name)
        t = agg.setdefault(k, [0, 0.0, 0.0, 1e30])
        d = (e - s) / 1e6
        t[0] += 1
        t[1] += d
        t[2] = max(t[2], d)
        t[3] = min(t[3], d)
    total = sum(v[1] for v in agg.values())
    out = sorted(agg.items(), key=lambda kv: -kv[1][1])
    w = csv.writer(open(a.csv, "w", newline="")) if a.csv else None
    if w:
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
    for k, (n, tot, mx, mn) in out:
        print(f"{tot:10.2f} ms {n:6d} calls avg {tot / n:9.3f} ms  {100 * tot / total:5.1f}%  {k}")
        if w:
            w.writerow([k, n, int(tot * 1e6), int(tot * 1e6 / n), 100 * tot / total, int(mn * 1e6), int(mx * 1e6)])
    span = (rows[-1][2] - rows[0][1]) / 1e6
    print(f"kernel busy {total:.1f} ms over span {span:.1f} ms")
    if a.timeline:
        prev = rows[0][1]
        for name, s, e in rows:
            print(f"{(s - rows[0][1]) / 1e6:10.3f} gap {(s - prev) / 1e6:8.3f} dur {(e - s) / 1e6:8.3f} {short(name)}")
            prev = e


if __name__ == "__main__":
    sys.exit(main())

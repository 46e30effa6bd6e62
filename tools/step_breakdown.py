#!/usr/bin/env python3
"""Device time by kernel class inside the timed proof of `bench.py --warmup 1 --steps 1`, from a
rocprofv3 --kernel-trace CSV (tools/prof_round.sh writes gpurun_out/r1_trace/**/run_kernel_trace.csv).

The timed proof starts at the second launch of its first kernels (k_copy_to_mont on the main lane,
the B plan's k_digits_c on the aux lane) and lasts the bench's own ms_per_step (bench JSON of the same
profiled run).  Kernel durations of both lanes are summed per class, so the total exceeds the wall time
where the lanes overlap.
"""
import csv
import glob
import json
import sys

CLASSES = [
    ("G1 accumulation (H, L, A, B_G1)", ("k_accum_level0<mi::fq_t>",)),
    ("G2 accumulation (B_G2 + second level)", ("k_accum_level0<mi::fq2_t>",)),
    ("bucket reduction (G1 + G2)", ("k_bucket_reduce", "k_seg_fold", "k_sum_groups", "k_tree_level",
                                    "k_bucket_affine")),
    ("NTT (7 transforms)", ("k_ntt_pass",)),
    ("digits + sort + bounds", ("k_digits", "onesweep", "k_bounds", "k_l2_digits", "radix_sort",
                                "k_chunk", "k_end_to_cnt", "k_flag_multi", "k_tree_count", "k_tree_heads")),
]


def main(path, bench_json):
    f = glob.glob(path + "/**/run_kernel_trace.csv", recursive=True)[0]
    rows = [(r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in csv.DictReader(open(f))]
    rows.sort(key=lambda r: r[1])

    def nth(sub, k):
        hits = [r for r in rows if sub in r[0]]
        return hits[k - 1] if len(hits) >= k else None

    t0 = min(nth("k_copy_to_mont", 2)[1], nth("k_digits_c(", 2)[1])
    t1 = t0 + int(json.load(open(bench_json))["ms_per_step"] * 1e6)
    acc = {name: 0.0 for name, _ in CLASSES}
    acc["rest"] = 0.0
    for name, s, e in rows:
        if s < t0 or s >= t1:
            continue
        ms = (e - s) / 1e6
        for cname, keys in CLASSES:
            if any(k in name for k in keys):
                acc[cname] += ms
                break
        else:
            acc["rest"] += ms
    for k, v in acc.items():
        print(f"| {k} | {v:.0f} |")
    print(f"| **sum of kernel time** | **{sum(acc.values()):.0f}** |")
    print(f"| **wall (bench ms_per_step)** | **{(t1 - t0) / 1e6:.0f}** |")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/r1_trace",
         sys.argv[2] if len(sys.argv) > 2 else "gpurun_out/r1_trace.json")

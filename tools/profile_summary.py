#!/usr/bin/env python3
"""Summarise rocprofv3 output of a bench.py run into profiles/<tag>_summary.json (+ copy the
kernel_stats CSV).

    python tools/profile_summary.py --tag r01 --trace gpurun_out/r1_trace \
        --fetch gpurun_out/r1_fetch --write gpurun_out/r1_write --bench-json gpurun_out/r1_trace.json

Traffic (MI355X_MICROARCH.md, HBM / rocprofv3): HBM bytes = FETCH_SIZE + WRITE_SIZE (KiB units,
x 1024), collected in separate --pmc passes.  On gfx950 FETCH_SIZE reads exactly 1/2 of the bytes
of wide (16 B/lane) coalesced reads, so the fetch side is reported both raw and x2-corrected; the
gathers of the MSM accumulation kernel are 16-byte-per-lane loads of 112-byte points, so the
corrected figure is the one used.  Per-launch bytes are divided by the points that launch processed
(reconstructed from the bench's deterministic launch order) to give bytes per point.
"""
import argparse
import csv
import glob
import json
import os
import shutil

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
A_PLAN = "own"  # set by main(): how the profiled proofs planned A (g1_launch_points)


def _one(path, pattern):
    hits = glob.glob(os.path.join(path, "**", pattern), recursive=True)
    if not hits:
        raise FileNotFoundError(f"{pattern} under {path}")
    return hits[0]


def kernel_stats(trace_dir):
    rows = list(csv.DictReader(open(_one(trace_dir, "*kernel_stats.csv"))))
    out = []
    for r in rows:
        out.append({"kernel": r["Name"], "calls": int(r["Calls"]), "total_ms": float(r["TotalDurationNs"]) / 1e6,
                    "avg_ms": float(r["AverageNs"]) / 1e6, "percent": float(r["Percentage"])})
    return out


def counter_per_dispatch(pmc_dir, counter, kernel_substr):
    rows = list(csv.DictReader(open(_one(pmc_dir, "*counter_collection.csv"))))
    vals = []
    for r in rows:
        if r["Counter_Name"] == counter and kernel_substr in r["Kernel_Name"]:
            vals.append((int(r["Dispatch_Id"]), float(r["Counter_Value"])))
    vals.sort()
    return [v for _, v in vals]


def step_launch_avg_ms(trace_dir, kernel_substr, bench):
    """Average duration of the dominant kernel over the launches of the TIMED steps only (the
    launch order is warmup proves, timed proves, standalone MSMs), to set beside bench.py's own
    HIP-event average ("roofline.avg_launch_ms")."""
    rows = [r for r in csv.DictReader(open(_one(trace_dir, "*kernel_trace.csv"))) if kernel_substr in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rows]
    lo, hi = 4 * bench["warmup"], 4 * (bench["warmup"] + bench["steps"])
    return sum(d[lo:hi]) / max(hi - lo, 1), [round(x, 3) for x in d]


def g1_launch_points(bench):
    """points processed by each k_accum_level0<G1> launch of `bench.py --warmup W --steps K` in submission
    (dispatch-id) order: per prove H, L, A, B_G1 (the warm-up and timed proves, then the one-lane proof of
    valu_roofline.one_lane when the line has it); then the standalone MSM (1 warm + msm_reps)."""
    cfg = bench["config"]
    per_prove = [cfg["domain"] - 1, cfg["num_aux"], cfg["a_query"], cfg["b_query"]]
    if A_PLAN in ("derived", "shared"):  # A as its aux part over L's plan plus a small MSM over the inputs' points
        per_prove = [cfg["domain"] - 1, cfg["num_aux"], cfg["a_query"] - cfg["num_inputs"], cfg["b_query"],
                     cfg["num_inputs"]]
    one_lane = (bench.get("valu_roofline") or {}).get("one_lane") or {}
    proves = bench["warmup"] + bench["steps"] + (1 if "avg_launch_ms" in one_lane else 0)
    msm = [bench["msm_g1_points"]] * (1 + bench.get("msm_reps", 1))
    return per_prove * proves + msm


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag", required=True)
    ap.add_argument("--trace", required=True)
    ap.add_argument("--fetch")
    ap.add_argument("--write")
    ap.add_argument("--bench-json", required=True)
    ap.add_argument("--kernel", default="k_accum_level0<mi::fq_t>")
    ap.add_argument("--command-file", help="the profiled bench command (tools/prof_round.sh writes <tag>_command.txt)")
    ap.add_argument("--a-plan", choices=["own", "shared", "derived"],
                    help="A's plan in the profiled proofs (default: the bench line's config.a_plan, else own)")
    args = ap.parse_args()
    bench = json.loads(open(args.bench_json).read().strip().splitlines()[-1])
    global A_PLAN
    A_PLAN = args.a_plan or bench["config"].get("a_plan") or "own"
    bench.setdefault("msm_reps", 1)
    cmd = open(args.command_file).read().strip() if args.command_file else "python3 bench.py (see tools/prof_round.sh)"
    out = {"tag": args.tag, "command": "rocprofv3 --kernel-trace --stats / --pmc FETCH_SIZE / --pmc WRITE_SIZE -- " + cmd,
           "workload": bench["config"]["workload"], "bench_value_under_profiler": bench["value"],
           "kernels": kernel_stats(args.trace)}
    try:  # the source revision the profiled build came from (bench.py reports it as roofline.traffic_detail)
        import subprocess

        out["commit"] = subprocess.check_output(["git", "-C", ROOT, "rev-parse", "--short=12", "HEAD"]).decode().strip()
    except Exception:
        out["commit"] = None
    dom = next(k for k in out["kernels"] if args.kernel in k["kernel"])
    out["dominant_kernel"] = {"name": args.kernel, "calls": dom["calls"], "avg_ms": dom["avg_ms"],
                              "total_ms": dom["total_ms"]}
    try:
        avg, per = step_launch_avg_ms(args.trace, args.kernel, bench)
        out["dominant_kernel"].update({"timed_step_launch_avg_ms": avg, "launch_ms": per,
                                       "bench_hip_event_avg_launch_ms": bench["roofline"]["avg_launch_ms"]})
    except FileNotFoundError:
        pass
    if args.fetch and args.write:
        f = counter_per_dispatch(args.fetch, "FETCH_SIZE", args.kernel)
        w = counter_per_dispatch(args.write, "WRITE_SIZE", args.kernel)
        pts = g1_launch_points(bench)
        n = min(len(f), len(w), len(pts))
        fetch_b = sum(f[:n]) * 1024.0
        write_b = sum(w[:n]) * 1024.0
        npts = float(sum(pts[:n]))
        out["dominant_kernel"].update({
            "pmc_launches": n,
            "fetch_bytes_raw_per_point": fetch_b / npts,
            "fetch_bytes_corrected_per_point": 2 * fetch_b / npts,
            "write_bytes_per_point": write_b / npts,
            "hbm_bytes_per_point": (2 * fetch_b + write_b) / npts,
            "algorithmic_bytes_per_point": 128.0,
        })
    os.makedirs(os.path.join(ROOT, "profiles"), exist_ok=True)
    dst = os.path.join(ROOT, "profiles", f"{args.tag}_summary.json")
    with open(dst, "w") as fh:
        json.dump(out, fh, indent=1)
    shutil.copy(_one(args.trace, "*kernel_stats.csv"), os.path.join(ROOT, "profiles", f"{args.tag}_kernel_stats.csv"))
    print(json.dumps(out["dominant_kernel"], indent=1))


if __name__ == "__main__":
    main()

#!/bin/bash
# Round-6 one-lane kernel traces (prove_lanes=1: every kernel alone on the chip, so its duration is its own):
#   winpost  one 32 GiB Window-PoSt partition (GPU witness + proof), breakdown by class and top kernels
#   c3       one config-3 proof (synthetic 2^26), breakdown by class (tools/lane_timeline.py) and top kernels
# Extra bench.py arguments (e.g. --tune msm_l0=128) follow the mode list after "--".
# usage: /usr/local/graft/bin/gpurun --timeout 900 -- bash tools/prof_r6.sh winpost c3 [-- --tune k=v]
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/prof_r6
mkdir -p $O
modes=(); extra=()
while [ $# -gt 0 ]; do
  if [ "$1" = "--" ]; then shift; extra=("$@"); break; fi
  modes+=("$1"); shift
done
QUIET=(--no-cpu-baseline --no-device-resident --tree-log-nodes 0 --sdr-log-labels 0 --config4-log-rows 0
       --stacked-log-nodes 0 --uniform-steps 0 --winning-log-nodes 0 --params-roundtrip 0 --tune prove_lanes=1)
for mode in "${modes[@]}"; do
  case $mode in
    winpost)
      B=(python3 bench.py --steps 1 --warmup 0 --log-rows 12 --msm-reps 1 --post-reps 2 --post-share-groups "" "${QUIET[@]}" "${extra[@]}")
      timeout -k 10 400 rocprofv3 --kernel-trace -d /tmp/wp -o run -- "${B[@]}" > $O/winpost_bench.json 2> $O/winpost_bench.err || { tail -5 $O/winpost_bench.err; exit 1; }
      python3 tools/winning_timeline.py /tmp/wp/run_results.db --reps 1 --md --top 25 > $O/winpost_timeline.md || exit 1
      cat $O/winpost_timeline.md ;;
    c3)
      B=(python3 bench.py --steps 3 --warmup 1 --msm-reps 1 --post-sectors 0 "${QUIET[@]}" "${extra[@]}")
      timeout -k 10 400 rocprofv3 --kernel-trace -d /tmp/c3 -o run -- "${B[@]}" > $O/c3_bench.json 2> $O/c3_bench.err || { tail -5 $O/c3_bench.err; exit 1; }
      python3 tools/lane_timeline.py /tmp/c3/run_results.db > $O/c3_timeline.txt || exit 1
      python3 - /tmp/c3/run_results.db > $O/c3_top.md <<'PY' || exit 1
import collections, sqlite3, sys
sys.path.insert(0, "tools")
from rocpd_summary import short
db = sqlite3.connect(sys.argv[1])
rows = list(db.execute("select name, start, end from kernels order by start"))
marks = [r[1] for r in rows if "k_copy_to_mont" in r[0]]
t0, t1 = marks[-2], marks[-1]
agg = collections.defaultdict(lambda: [0, 0.0])
for n, s, e in rows:
    if t0 <= s < t1:
        agg[short(n)][0] += 1
        agg[short(n)][1] += (e - s) / 1e6
print("| kernel | launches | device ms |\n|---|---|---|")
for n, (c, ms) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:30]:
    print(f"| `{n[:70]}` | {c} | {ms:.2f} |")
PY
      cat $O/c3_timeline.txt; cat $O/c3_top.md ;;
    *) echo "unknown mode $mode"; exit 2 ;;
  esac
done

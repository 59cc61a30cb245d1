#!/bin/bash
# A/B of the literal BodyEfforts kernel (k_pose_efforts_epoch) over variant
# libraries: rocprofv3 kernel stats of the C4 bench (2,000 epochs, compressed
# drop-out cycle: 7 efforts epochs), the efforts kernel's average duration and
# the bench's ensemble statistics (equal NEES = the same results).
# Usage (repo root, on the box): bash tools/ab_eff.sh TAG ROUNDS v1 v2 ...   (v = libuwvk_v.so)
set -u
TAG=$1; ROUNDS=$2; shift 2
OUT=$PWD/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for r in $(seq 1 $ROUNDS); do
  for v in "$@"; do
    export UWVK_LIB=$PWD/slam-uwv_kalman_filters_amd/libuwvk_$v.so
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/$v-$r" -o run -- \
      python3 bench.py --mode C4 --steps 2000 --warmup 5 --c4-cycle 0.3,0.1 --no-cpu-baseline \
      > "$OUT/$v-$r.json" 2> "$OUT/$v-$r.err" || { echo "$v failed"; tail -20 "$OUT/$v-$r.err"; exit 1; }
    python3 - "$OUT/$v-$r" "$v" <<'PY'
import csv, json, sys
d, v = sys.argv[1], sys.argv[2]
b = json.loads(open(d + ".json").read().strip().splitlines()[-1])
rows = list(csv.DictReader(open(d + "/run_kernel_stats.csv")))
eff = [r for r in rows if "efforts_epoch" in r["Name"]]
for r in eff:
    print(v, r["Name"][:60], "calls", r["Calls"], "avg %.3f ms" % (float(r["AverageNs"]) / 1e6))
print(v, "C4 %.2f M steps/s" % (b["value"] / 1e6), "nees", b["ensemble"])
PY
  done
done

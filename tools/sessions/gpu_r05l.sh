#!/bin/bash
# r05l: three update-phase VALU cuts as A/B variants of the PSP unit:
#   psel  P = H L_a^T per row with H's entries as operands, one select of the lane's row (PSP_PSEL)
#   pr    + R's rows through the staging area instead of lane-indexed select chains (PSP_RLDS)
#   prh   + the measurement Jacobian kept in VGPRs (no readlane / SGPR spill) (PSP_HVGPR)
# Parity of the widest variant (GPU parity, efforts, SO3-side tests under
# UWVK_LIB), then interleaved C3 A/B rounds against the shipped build.
set -u
OUT=$PWD/gpurun_out/r05l
mkdir -p "$OUT"
PKGD=$PWD/slam-uwv_kalman_filters_amd
for v in prh pr; do
UWVK_LIB=$PKGD/libuwvk_$v.so timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_efforts.py tests/test_gpu_so3_side.py \
  -q -m gpu -x --timeout 200 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_$v.txt" 2>&1 || { tail -30 "$OUT/pytest_$v.txt"; exit 1; }
echo "$v: $(tail -1 $OUT/pytest_$v.txt)"
done
bash tools/ab_variants.sh r05l 3 psel pr prh | tee "$OUT/summary.txt"
# instruction-cache counters of the shipped C3 kernel (never measured before):
# the counter list first, then one --pmc pass with the SQC ones it has
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -s KILL 60 rocprofv3 -L > "$OUT/counters_list.txt" 2>&1 || true
CS=$(grep -o "SQC_ICACHE_[A-Z_]*\|SQ_IFETCH[A-Z_]*" "$OUT/counters_list.txt" | sort -u | grep -v "_sum\|_LEVEL" | head -4 | tr '\n' ' ')
echo "icache counters: $CS"
if [ -n "$CS" ]; then
  timeout -s KILL 90 rocprofv3 --pmc $CS SQ_WAVES SQ_INSTS_VALU --output-format csv -d "$OUT/icache" -o run -- \
    python3 bench.py --steps 20 --warmup 2 --no-cpu-baseline > "$OUT/icache.log" 2>&1 || { tail -5 "$OUT/icache.log"; exit 1; }
  python3 - "$OUT/icache/run_counter_collection.csv" <<'PY'
import csv, sys
rows = [r for r in csv.DictReader(open(sys.argv[1])) if "psp_epoch" in r["Kernel_Name"]]
disp = {}
for r in rows:
    disp.setdefault(r["Dispatch_Id"], {}).setdefault(r["Counter_Name"], 0.0)
    disp[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
d = max(disp, key=lambda k: disp[k].get("SQ_INSTS_VALU", 0))
for c, v in sorted(disp[d].items()):
    print("%-28s %16.6g" % (c, v))
PY
fi

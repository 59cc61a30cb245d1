#!/bin/bash
# A/B of the last-generation spreading (bench.py --tail-slots -1 vs 0) at 20 and
# 200 epochs, interleaved twice: kernel ms per launch (HIP events)
set -u
OUT=$PWD/gpurun_out/ab_tail
mkdir -p "$OUT"
for rep in 1 2; do
  for s in 20 200; do
    for t in -1 0; do
      n="t${t}-s${s}-r${rep}"
      timeout -k 10 200 python bench.py --steps $s --warmup 5 --no-cpu-baseline --tail-slots $t > "$OUT/$n.json" 2> "$OUT/$n.err" || { echo "$n failed"; tail -5 "$OUT/$n.err"; exit 1; }
      python -c "import json; d=json.load(open('$OUT/$n.json')); t=d['timing']; print('$n', '%.2fM' % (d['value']/1e6), 'kernel %.3f ms' % t['kernel_ms'])"
    done
  done
done

#!/bin/bash
# Short-window gap decomposition: the 20-epoch C3 line with its DVL update
# (default alignment) and with the window moved 100 epochs off it, interleaved.
set -u
OUT=$PWD/gpurun_out/ab_dvl
mkdir -p "$OUT"
for i in 1 2 3; do
  for off in 0 100; do
    UWVK_BENCH_WINDOW_OFFSET=$off timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/off$off-$i.json" 2> "$OUT/off$off-$i.err" || { tail -5 "$OUT/off$off-$i.err"; exit 1; }
    python -c "import json; d=json.load(open('$OUT/off$off-$i.json')); t=d['timing']; print('offset $off', 'dvl', d['config']['dvl_epochs_in_window'], '%.2fM' % (d['value']/1e6), 'kernel %.3f ms' % t['kernel_ms'])"
  done
done

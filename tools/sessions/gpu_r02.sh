#!/bin/bash
# Round-2 GPU session: new parity tests (surface, sharded), the driver-shape
# bench line, a world-size-1 torchrun (RCCL) bench line, a CPU-share probe and
# one SQ/GRBM counter pass.  Usage (repo root, on the box): bash tools/gpu_r02.sh TAG [TESTS...]
set -u
TAG=${1:-r02}
shift || true
TESTS=${*:-tests/test_gpu_surface.py tests/test_distributed.py}
OUT=$PWD/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
python3 -c "import os; print('affinity', len(os.sched_getaffinity(0)), 'cpu_count', os.cpu_count())" > "$OUT/cpu_probe.txt"
cat /sys/fs/cgroup/cpu.max >> "$OUT/cpu_probe.txt" 2>&1
timeout -k 10 900 python -u -m pytest $TESTS -v -m gpu --timeout 900 --timeout-method thread -p no:cacheprovider \
  > "$OUT/pytest_gpu.log" 2>&1
echo "pytest rc=$?" >> "$OUT/pytest_gpu.log"
tail -5 "$OUT/pytest_gpu.log"
grep -q "FAILED\|Error" "$OUT/pytest_gpu.log" && grep -E "FAILED|^E " "$OUT/pytest_gpu.log" | head -40
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > "$OUT/bench_s20.json" 2> "$OUT/bench_s20.err" || { tail -20 "$OUT/bench_s20.err"; exit 1; }
cut -c1-400 "$OUT/bench_s20.json"
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29611 \
  bench.py --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/bench_torchrun1.json" 2> "$OUT/bench_torchrun1.err" || { tail -20 "$OUT/bench_torchrun1.err"; exit 1; }
cut -c1-300 "$OUT/bench_torchrun1.json"
timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_WAVES SQ_CYCLES SQ_INSTS_VALU GRBM_GUI_ACTIVE GRBM_COUNT \
  --output-format csv -d "$OUT/pmc_busy" -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/pmc_busy.log" 2>&1 || { tail -20 "$OUT/pmc_busy.log"; exit 1; }
echo done

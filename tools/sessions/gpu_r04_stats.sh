#!/bin/bash
# r04 end: rocprofv3 kernel-trace summaries of the current C2 and C4 runs
# (kernel stats next to the bench line measured under the profiler).
set -o pipefail
O=gpurun_out/stats; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c2 -o run -- \
  python3 bench.py --mode C2 --steps 2000 --warmup 5 --no-cpu-baseline > $O/bench_c2_traced.json 2> $O/c2.err || { tail -5 $O/c2.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c4 -o run -- \
  python3 bench.py --mode C4 --steps 2000 --warmup 5 --no-cpu-baseline > $O/bench_c4_traced.json 2> $O/c4.err || { tail -5 $O/c4.err; exit 1; }
find $O/c2 -name "*kernel_stats*" -exec cp {} $O/kernel_stats_c2.csv \;
find $O/c4 -name "*kernel_stats*" -exec cp {} $O/kernel_stats_c4.csv \;
echo done

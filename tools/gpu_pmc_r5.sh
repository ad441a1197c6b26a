#!/bin/bash
# Round-5 counter passes at config 3: the faithful sorted, radix and uniform
# passes (tools/gpu_pmc_faithful.sh: SQ counters, FETCH_SIZE, WRITE_SIZE, each
# pass in its own run).  usage: tools/gpu_pmc_r5.sh OUT
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${1:-pmc5}
for mode in sorted radix uniform; do
  PROF_SHAPE=config3 PROF_REPS=3 bash tools/gpu_pmc_faithful.sh "$OUT/$mode" $mode || exit $?
  echo "$mode done"
done
# the bench command under a kernel trace (profiles/: the hot kernel's average
# duration agrees with the bench line's HIP-event figure)
mkdir -p gpurun_out/$OUT/bench_trace
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$OUT/bench_trace -o run -- python bench.py > gpurun_out/$OUT/bench_trace.json 2> gpurun_out/$OUT/bench_trace.err || exit $?
tail -1 gpurun_out/$OUT/bench_trace.json | cut -c1-300

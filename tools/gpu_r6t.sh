#!/bin/bash
# Kernel traces of the faithful config-3 passes, one source per run (sorted,
# radix), for the per-kernel budget.  usage: tools/gpu_r6t.sh OUT
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r6t}
mkdir -p "$OUT"
for src in sorted radix; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$src" -o run --output-format csv -- \
    python tools/fa_time.py 4096 8 28 --only $src > "$OUT/$src.log" 2>&1 \
  && python tools/stats_summary.py "$OUT/prof_$src/run_kernel_stats.csv" > "$OUT/stats_$src.txt" \
  && echo "== $src" && tail -1 "$OUT/$src.log" && head -14 "$OUT/stats_$src.txt" || exit 1
done

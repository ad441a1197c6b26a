#!/bin/bash
# Round-5 development session: the uniform source (tests, pass and part timings, kernel stats)
# and the faithful group's fixed cost (group_time, a kernel trace split per call).
# usage: tools/gpu_r5c.sh OUT
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r5c}
mkdir -p "$OUT"
bash tools/gpu_uni_dev.sh "${1:-r5c}" || exit 1
echo "== group times"
timeout -k 10 300 python tools/group_time.py generated 5 > "$OUT/group_gen.json" 2>&1 && cat "$OUT/group_gen.json" \
&& timeout -k 10 300 python tools/group_time.py uniform 5 > "$OUT/group_uni.json" 2>&1 && cat "$OUT/group_uni.json" \
&& timeout -k 10 300 rocprofv3 --kernel-trace -d "$OUT/gprof" -o run --output-format csv -- python tools/group_time.py generated 2 \
  > "$OUT/gprof.log" 2>&1 && python tools/trace_span.py "$OUT/gprof/run_kernel_trace.csv" 300 > "$OUT/gspan.txt" && cat "$OUT/gspan.txt"

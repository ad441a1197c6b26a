#!/bin/bash
# A development session on the faithful pipeline: its GPU tests, the pass
# times of every source at BASELINE configs 2 and 3 (tools/fa_time.py), and a
# rocprofv3 kernel trace of the config-3 passes.  usage: tools/gpu_fa_dev.sh OUT
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-fadev}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_faithful_wide.py \
  tests/test_gpu_uniform.py tests/test_group_capi.py tests/test_gpu.py -k "faithful or shard or group or uniform or r10 or dump" \
  > "$OUT/pytest.log" 2>&1; rc=$?; tail -3 "$OUT/pytest.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/fa_time.py 1024 8 24 4096 8 28 > "$OUT/fa_time.json" 2>&1 && grep '{' "$OUT/fa_time.json" \
&& timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python tools/fa_time.py 4096 8 28 \
  > "$OUT/prof.log" 2>&1 && python tools/stats_summary.py "$OUT/prof/run_kernel_stats.csv" > "$OUT/stats.txt" && head -24 "$OUT/stats.txt"

#!/bin/bash
# Round-5 check: the faithful and group GPU tests, then the faithful pass times and the group call times.
# usage: tools/gpu_r5d.sh OUT
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r5d}
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_group_capi.py \
  tests/test_gpu_uniform.py tests/test_gpu_faithful_wide.py tests/test_gpu.py -k "faithful or shard or group or uniform or r10 or dump or replay" \
  > "$OUT/pytest.log" 2>&1; rc=$?; tail -3 "$OUT/pytest.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/fa_time.py 4096 8 28 > "$OUT/fa_time.json" 2>&1 && cat "$OUT/fa_time.json" \
&& timeout -k 10 300 python tools/group_time.py generated 5 > "$OUT/group_gen.json" 2>&1 && tail -1 "$OUT/group_gen.json" \
&& timeout -k 10 300 python tools/group_time.py uniform 5 > "$OUT/group_uni.json" 2>&1 && tail -1 "$OUT/group_uni.json"

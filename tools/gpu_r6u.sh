#!/bin/bash
# Round 6: the uniform group pass captured and replayed.  Group + uniform GPU
# tests, then the group times (uniform, generated).  usage: tools/gpu_r6u.sh OUT
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r6u}
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_group_capi.py \
  tests/test_gpu_uniform.py > "$OUT/pytest.log" 2>&1; rc=$?; tail -3 "$OUT/pytest.log"; [ $rc -eq 0 ] || exit $rc
for src in uniform generated; do
  timeout -k 10 300 python tools/group_time.py $src 7 > "$OUT/group_$src.json" 2> "$OUT/group_$src.err" || { tail -3 "$OUT/group_$src.err"; exit 1; }
  tail -1 "$OUT/group_$src.json"
done

#!/bin/bash
# Round 6, first session: smoke, the group tests (the config-3 any-order case
# at 1/2/8 shards on the count-free sort: r5p's sequence), the r5p command
# itself (group_time.py any_order), then every GPU test.
# usage: tools/gpu_r6a.sh OUT   (results under gpurun_out/OUT)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r6a}
mkdir -p "$OUT"
echo "== smoke" && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 && tail -1 "$OUT/smoke.log" \
&& echo "== group tests" && timeout -k 10 600 python -u -m pytest tests/test_group_capi.py -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest_group.log" 2>&1; rc=$?; tail -3 "$OUT/pytest_group.log"; [ $rc -eq 0 ] \
&& echo "== group_time any_order" && timeout -k 10 300 python tools/group_time.py any_order 5 > "$OUT/group_any_order.json" 2>&1; rc=$?; tail -1 "$OUT/group_any_order.json"; [ $rc -eq 0 ] \
&& echo "== pytest -m gpu" && timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1; rc=$?; tail -3 "$OUT/pytest_gpu.log"; exit $rc

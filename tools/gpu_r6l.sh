#!/bin/bash
# Round 6: a library with no scratch-requesting kernel.  r5p's command
# (group_time any_order) three times, the faithful config-3 times, the new
# and uniform tests, smoke, every GPU test.  usage: tools/gpu_r6l.sh OUT
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r6l}
mkdir -p "$OUT"
for k in 1 2 3 4; do
  timeout -k 10 300 python tools/group_time.py any_order 5 > "$OUT/any_order_$k.json" 2>&1 || { tail -2 "$OUT/any_order_$k.json"; exit 1; }
  tail -1 "$OUT/any_order_$k.json"
done
echo "== fa_time config 3" && timeout -k 10 300 python tools/fa_time.py 4096 8 28 > "$OUT/fa_time.json" 2>&1; rc=$?; tail -1 "$OUT/fa_time.json"; [ $rc -eq 0 ] || exit $rc
echo "== new + uniform tests"
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu.py::test_pair_sort_shapes_vs_oracle tests/test_gpu_uniform.py tests/test_group_capi.py > "$OUT/pytest_new.log" 2>&1; rc=$?; tail -3 "$OUT/pytest_new.log"; [ $rc -eq 0 ] || exit $rc
echo "== smoke" && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 && tail -1 "$OUT/smoke.log" \
&& echo "== pytest -m gpu" && timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1; rc=$?; tail -3 "$OUT/pytest_gpu.log"; exit $rc

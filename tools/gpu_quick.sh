#!/bin/bash
# Short GPU iteration: the named GPU test files (default: all -m gpu tests), then the bench line.
# usage: tools/gpu_quick.sh OUT [pytest selection...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-quick}
shift
SEL=${@:-tests}
mkdir -p "$OUT"
echo "== pytest -m gpu $SEL" && timeout -k 10 900 python -u -m pytest $SEL -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1; rc=$?; tail -4 "$OUT/pytest_gpu.log"; [ $rc -eq 0 ] \
&& echo "== bench" && timeout -k 10 600 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"; rc=$?; tail -c 4000 "$OUT/bench.json"; tail -5 "$OUT/bench.err"; exit $rc

#!/bin/bash
# Short GPU iteration: parity tests, the bench line (no side measurements), ablation.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-quick}
mkdir -p "$OUT"
echo "== pytest -m gpu" && timeout -k 10 900 python -m pytest tests -m gpu -x -q > "$OUT/pytest_gpu.log" 2>&1; rc=$?; tail -5 "$OUT/pytest_gpu.log"; [ $rc -eq 0 ] \
&& echo "== bench" && timeout -k 10 600 python bench.py --no-extras --no-cpu-baseline > "$OUT/bench.json" 2> "$OUT/bench.err" && cat "$OUT/bench.json" \
&& echo "== ablate" && timeout -k 10 300 python tools/ablate.py > "$OUT/ablate.jsonl" 2> "$OUT/ablate.err" && cat "$OUT/ablate.jsonl"

#!/bin/bash
# Faithful-mode iteration: its GPU parity tests, then the bench's side measurements.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-faith}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -k "faithful" --timeout 300 --timeout-method thread > "$OUT/pytest_faith.log" 2>&1; rc=$?; tail -3 "$OUT/pytest_faith.log"; [ $rc -eq 0 ] \
&& timeout -k 10 400 python bench.py --steps 50 --warmup 5 --no-cpu-baseline > "$OUT/bench.json" 2> "$OUT/bench.err" && python -c "
import json; d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1]); print(json.dumps(d['faithful'])); print(json.dumps(d['fulltrace']))"

#!/bin/bash
# all GPU tests, the bench line, and a kernel trace of the faithful side measurements
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r2c}
mkdir -p "$OUT"
echo "== pytest -m gpu" && timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1; rc=$?; tail -4 "$OUT/pytest_gpu.log"; [ $rc -eq 0 ] \
&& echo "== bench" && timeout -k 10 600 python bench.py --no-cpu-baseline > "$OUT/bench.json" 2> "$OUT/bench.err" && python -c "
import json; d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1]); print(d['value'], d['roofline']['frac']); print(json.dumps(d['faithful'])); print(json.dumps(d['end_to_end']))" \
&& echo "== trace" && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python bench.py --no-cpu-baseline --steps 20 > "$OUT/prof.log" 2>&1 \
&& python tools/stats_summary.py "$OUT/prof/run_kernel_stats.csv" | head -30

#!/bin/bash
# One GPU-box session: smoke, GPU parity tests, bench, rocprofv3 kernel trace.
# Each GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r01}
mkdir -p "$OUT"
echo "== smoke" && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 && tail -2 "$OUT/smoke.log" \
&& echo "== pytest -m gpu" && timeout -k 10 900 python -m pytest tests -m gpu -x -q > "$OUT/pytest_gpu.log" 2>&1; rc=$?; tail -15 "$OUT/pytest_gpu.log"; [ $rc -eq 0 ] \
&& echo "== bench" && timeout -k 10 600 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" && cat "$OUT/bench.json" \
&& echo "== rocprofv3 kernel trace" && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python bench.py > "$OUT/prof.log" 2>&1 && find "$OUT/prof" -name "*kernel_stats.csv" | wc -l
[ $? -eq 0 ] && echo "== ablate" && timeout -k 10 300 python tools/ablate.py > "$OUT/ablate.jsonl" 2> "$OUT/ablate.err" && cat "$OUT/ablate.jsonl" \
&& echo "== pmc" && bash tools/prof_round.sh "${1:-r01}/pmc" noablate > "$OUT/pmc.log" 2>&1; tail -30 "$OUT/pmc.log"

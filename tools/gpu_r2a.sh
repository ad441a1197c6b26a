#!/bin/bash
# Round-2 GPU session: parity tests, the bench line (config 3), the rocprofv3
# kernel trace of the same command, PMC passes at 2^28, ablation.  Every GPU
# step has its own time limit; the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r2a}
mkdir -p "$OUT"
echo "== pytest -m gpu" && timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1; rc=$?; tail -5 "$OUT/pytest_gpu.log"; [ $rc -eq 0 ] \
&& echo "== bench" && timeout -k 10 600 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" && cat "$OUT/bench.json" \
&& echo "== rocprofv3 kernel trace" && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python bench.py --no-cpu-baseline > "$OUT/prof.log" 2>&1 \
&& echo "== pmc" && for c in FETCH_SIZE WRITE_SIZE "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS"; do \
     timeout -k 10 120 rocprofv3 --pmc $c --output-format csv -d "$OUT/pmc_$(echo $c | cut -d' ' -f1)" -o run -- python tools/prof_kernel.py > "$OUT/pmc_$(echo $c | cut -d' ' -f1).log" 2>&1 || exit 1; done \
&& echo "== ablate" && timeout -k 10 300 python tools/ablate.py > "$OUT/ablate.jsonl" 2> "$OUT/ablate.err" && cat "$OUT/ablate.jsonl"

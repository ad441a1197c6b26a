#!/bin/bash
# Counter passes (FETCH_SIZE / WRITE_SIZE / SQ) of the faithful pass at config 3
# for the radix (any-order lists, bucket sort inside the pass) and uniform
# sources.  usage: tools/gpu_pmc_sources.sh OUT
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${1:-pmcs}
mkdir -p "gpurun_out/$OUT"
for m in radix uniform; do
  PROF_SHAPE=config3 PROF_REPS=3 bash tools/gpu_pmc_faithful.sh "$OUT/$m" "$m" > "gpurun_out/$OUT/$m.log" 2>&1 || { echo "$m failed"; tail -5 "gpurun_out/$OUT/$m.log"; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/$OUT/$m/pmc_faithful.json')); print('$m', d['hbm_bytes_per_pass'], d['hbm_bytes_per_sample'])"
done

#!/bin/bash
# The round's closing GPU session: tools/gpu_full_round.sh (smoke, every GPU
# test, the bench line, its kernel trace, config 2 / config 4 lines), then the
# faithful counter passes at configs 3 and 2, then a two-rank gloo rehearsal of
# bench.py --gpus 2 (both ranks on this one GPU; the collective and the
# key-range-sharded faithful side lines).  usage: tools/gpu_final_round.sh OUT
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${1:-final}
bash tools/gpu_full_round.sh "$OUT" || exit 1
echo "== pmc faithful config 3" && PROF_SHAPE=config3 bash tools/gpu_pmc_faithful.sh "$OUT/pmcf3" sorted > "gpurun_out/$OUT/pmcf3.log" 2>&1 \
  && python -c "import json; print(json.load(open('gpurun_out/$OUT/pmcf3/pmc_faithful.json'))['hbm_bytes_per_pass'])" || exit 1
echo "== pmc faithful config 2" && bash tools/gpu_pmc_faithful.sh "$OUT/pmcf2" sorted > "gpurun_out/$OUT/pmcf2.log" 2>&1 \
  && python -c "import json; print(json.load(open('gpurun_out/$OUT/pmcf2/pmc_faithful.json'))['hbm_bytes_per_pass'])" || exit 1
echo "== gloo x2 rehearsal" && timeout -k 10 400 python bench.py --gpus 2 --backend gloo --steps 10 --warmup 2 --no-cpu-baseline \
  > "gpurun_out/$OUT/bench_gloo2.json" 2> "gpurun_out/$OUT/bench_gloo2.err" \
  && python -c "
import json; d=json.loads(open('gpurun_out/$OUT/bench_gloo2.json').read().strip().splitlines()[-1])
print(d['value'], d['n_gpus'], json.dumps(d.get('collective')), json.dumps(d.get('faithful_sharded')))"

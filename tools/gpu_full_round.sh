#!/bin/bash
# One GPU-box session on the final tree: smoke, every GPU test, the full bench line, a
# rocprofv3 kernel trace of the bench, and the config 2 / config 4 bench lines.
# usage: tools/gpu_full_round.sh OUT   (results under gpurun_out/OUT)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-full}
mkdir -p "$OUT"
echo "== smoke" && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 && tail -2 "$OUT/smoke.log" \
&& echo "== pytest -m gpu" && timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1; rc=$?; tail -4 "$OUT/pytest_gpu.log"; [ $rc -eq 0 ] \
&& echo "== bench" && timeout -k 10 600 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" && python -c "
import json; d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1]); print(d['value'], d['roofline']['frac'], d['roofline']['traffic']); print(json.dumps(d['faithful_config3'])); print(json.dumps(d['cpu_baseline']))" \
&& echo "== trace" && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python bench.py --no-cpu-baseline --steps 20 > "$OUT/prof.log" 2>&1 \
&& python tools/stats_summary.py "$OUT/prof/run_kernel_stats.csv" > "$OUT/stats.txt" && sed -n 1,30p "$OUT/stats.txt"
[ $? -eq 0 ] && echo "== config2/config4 bench lines" \
&& timeout -k 10 300 python bench.py --config config2 --no-extras --no-cpu-baseline > "$OUT/bench_config2.json" 2>> "$OUT/bench.err" \
&& timeout -k 10 300 python bench.py --config config4 --no-extras --no-cpu-baseline > "$OUT/bench_config4.json" 2>> "$OUT/bench.err" \
&& python -c "
import json
for c in ('config2','config4'):
    d=json.loads(open('$OUT/bench_'+c+'.json').read().strip().splitlines()[-1]); print(c, d['value'], d['ms_per_step'], d['roofline']['frac'])"

#!/bin/bash
# One GPU-box session: smoke, every GPU test, then the full bench line.
# usage: tools/gpu_session.sh OUT [pytest selection...]   (results under gpurun_out/OUT)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-session}
shift
SEL=${*:-tests}
mkdir -p "$OUT"
echo "== smoke" && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 && tail -1 "$OUT/smoke.log" \
&& echo "== pytest -m gpu $SEL" && timeout -k 10 900 python -u -m pytest $SEL -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1; rc=$?; tail -4 "$OUT/pytest_gpu.log"; [ $rc -eq 0 ] \
&& echo "== bench" && timeout -k 10 900 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" && python - "$OUT/bench.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(d["value"], d["ms_per_step"], d["roofline"]["frac"])
for k in ("faithful_config3", "faithful_pipeline", "capi_group"):
    print(k, json.dumps(d.get(k))[:1500])
PY

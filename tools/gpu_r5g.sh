#!/bin/bash
# Round-5 radix check: the sort and faithful GPU tests, the faithful pass
# times at config 3, and the radix pass's kernel trace.  usage: tools/gpu_r5g.sh OUT
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r5g}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_sort.py tests/test_group_capi.py \
  tests/test_gpu_faithful_wide.py tests/test_gpu.py -k "faithful or sort or radix or shard or group" > "$OUT/pytest.log" 2>&1; rc=$?; tail -3 "$OUT/pytest.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/fa_time.py 4096 8 28 > "$OUT/fa_time.json" 2>&1 && cat "$OUT/fa_time.json" \
&& PROF_SHAPE=config3 PROF_FAITH=radix PROF_REPS=5 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
  -d "$OUT/prof" -o run -- python tools/prof_faithful.py > "$OUT/prof.log" 2>&1 \
&& python - "$OUT" <<'PY'
import csv, glob, os, sys
f = glob.glob(os.path.join(sys.argv[1], "prof", "**", "*kernel_stats.csv"), recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:14]:
    print("%10.1f us %5s x %9.2f us  %s" % (float(r["TotalDurationNs"]) / 1e3, r["Calls"], float(r["AverageNs"]) / 1e3,
                                           r["Name"].split("(")[0].replace("void ", "").replace("pluss::", "")[:70]))
PY

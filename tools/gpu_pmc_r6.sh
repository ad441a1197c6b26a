#!/bin/bash
# Round 6 counter passes at config 3: the uniform, sorted and radix faithful
# passes (tools/gpu_pmc_faithful.sh per mode).  usage: tools/gpu_pmc_r6.sh OUT
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${1:-pmc6}
export PROF_SHAPE=config3 PROF_REPS=3
for mode in uniform sorted radix; do
  bash tools/gpu_pmc_faithful.sh "$OUT/$mode" $mode > /dev/null || { echo "mode $mode failed"; exit 1; }
  python - "gpurun_out/$OUT/$mode/pmc_faithful.json" $mode <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print(sys.argv[2], "B/sample", round(d.get("hbm_bytes_per_sample", 0), 3))
for k, v in d["per_kernel_per_pass_KB"].items():
    if "k_fa_local_lm" in k or "k_srt" in k:
        print("  ", k, "FETCH_KB", round(v.get("FETCH_SIZE", 0)), "WRITE_KB", round(v.get("WRITE_SIZE", 0)))
PY
done

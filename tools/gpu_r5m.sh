#!/bin/bash
# The radix probe (each call synchronised), then tools/gpu_r5g.sh.  usage: tools/gpu_r5m.sh OUT
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-r5m}
mkdir -p "$OUT"
timeout -k 10 240 python -u tools/radix_probe.py > "$OUT/probe.txt" 2>&1; rc=$?; tail -3 "$OUT/probe.txt"; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_r5g.sh "${1:-r5m}"

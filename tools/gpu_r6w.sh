#!/bin/bash
# Round 6: the uniform replay probe on the stage build (slice-check prints), then
# the group + uniform GPU tests and the group times.  usage: tools/gpu_r6w.sh OUT
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r6w}
mkdir -p "$OUT"
PLUSS_PROBE_LIB=stages PLUSS_STAGE_MODE=off timeout -k 10 300 python tools/uni_replay_probe.py > "$OUT/probe.log" 2>&1; rc=$?
grep -c "slice check" "$OUT/probe.log"; grep -v "^RCCL\|^HIP\|^ROCm\|^Hostname\|^Librccl\|slice check" "$OUT/probe.log" | tail -25
[ $rc -eq 0 ] && ! grep -q "ERROR\|DIFFERENT" "$OUT/probe.log" || exit 1
bash tools/gpu_r6u.sh "${1:-r6w}"

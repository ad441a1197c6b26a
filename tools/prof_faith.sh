#!/bin/bash
# rocprofv3 kernel traces of faithful mode (serial and concurrent) at config-2 size.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-pfaith}
mkdir -p "$OUT"
PROF_FAITH=serial timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/serial" -o run --output-format csv -- python tools/prof_side.py > "$OUT/serial.log" 2>&1 \
&& PROF_FAITH=concurrent timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/conc" -o run --output-format csv -- python tools/prof_side.py > "$OUT/conc.log" 2>&1
rc=$?
grep "faithful\|full trace" "$OUT/serial.log" "$OUT/conc.log"
exit $rc

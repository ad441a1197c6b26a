#!/bin/bash
# fa_time (radix) for several values of an environment variable.  usage: tools/gpu_ab2.sh OUT VAR v1 v2 ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/$1; VAR=$2; shift 2
mkdir -p "$OUT"
for v in "$@" "$@"; do
  env $VAR=$v timeout -k 10 300 python tools/fa_time.py --only radix 4096 8 28 > "$OUT/fa_$v.txt" 2>&1 || exit $?
  echo "$VAR=$v $(tail -1 $OUT/fa_$v.txt)"
done

#!/bin/bash
# A/B of an environment toggle on fa_time at config 3 (sorted, radix), each
# side twice.  usage: tools/gpu_ab.sh OUT VAR
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/$1
mkdir -p "$OUT"
for tag in 0 1 0 1; do
  if [ $tag = 0 ]; then
    timeout -k 10 300 python tools/fa_time.py --only sorted,radix 4096 8 28 > "$OUT/fa_$tag.txt" 2>&1 || exit $?
  else
    env $2=1 timeout -k 10 300 python tools/fa_time.py --only sorted,radix 4096 8 28 > "$OUT/fa_$tag.txt" 2>&1 || exit $?
  fi
  echo "$2=$tag $(tail -1 $OUT/fa_$tag.txt)"
done

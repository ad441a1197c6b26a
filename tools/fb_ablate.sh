#!/bin/bash
# Faithful bucket path: kernel times of k_fb_fused with the sort only (PLUSS_FB_ABL=1),
# the scan without the sort (=2), and the product (0); radix-sort path for comparison.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-fbabl}
mkdir -p "$OUT"
for a in 0 1 2; do
  PLUSS_FAITH_BUCKET=1 PLUSS_FB_ABL=$a timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$OUT/abl$a" -o run --output-format csv -- python tools/prof_side.py > "$OUT/abl$a.log" 2>&1 || exit 1
  grep "faithful" "$OUT/abl$a.log"
  grep "k_fb_\|k_faith" "$OUT/abl$a/run_kernel_stats.csv" | awk -F'","' '{split($1,a,"("); print "  abl'$a'", a[1], $2, $4}'
done
timeout -k 10 120 python tools/prof_side.py 2>&1 | grep faithful

#!/bin/bash
# tools/gpu_r5m.sh (probe, sort/faithful GPU tests, fa_time, radix kernel
# stats), then the radix pass's counter passes.  usage: tools/gpu_r5v.sh OUT
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_r5m.sh "$1" || exit $?
PROF_SHAPE=config3 PROF_REPS=3 bash tools/gpu_pmc_faithful.sh "$1/pmc_radix" radix

#!/bin/bash
# Rehearse the N>1 bench path on a one-GPU box: 2 ranks share cuda:0, dense vectors
# all-reduced over gloo (the round-end driver runs N=2..8 over RCCL on 8 GPUs).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-rehearse}
mkdir -p "$OUT"
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 2 --backend gloo > "$OUT/bench_n2_gloo.json" 2> "$OUT/bench_n2_gloo.err" && cat "$OUT/bench_n2_gloo.json"

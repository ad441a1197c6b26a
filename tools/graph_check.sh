set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/graph; mkdir -p $O
timeout -k 10 200 python bench.py --no-extras --no-cpu-baseline > $O/g20.json 2> $O/g20.err && \
timeout -k 10 200 python bench.py --no-extras --no-cpu-baseline --graph 0 > $O/eager.json 2> $O/eager.err && \
timeout -k 10 200 python bench.py --no-extras --no-cpu-baseline --steps 7 --warmup 2 > $O/g7.json 2> $O/g7.err && \
timeout -k 10 200 python -m torch.distributed.run --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29512 bench.py --no-extras --no-cpu-baseline --allreduce > $O/ar_g20.json 2> $O/ar_g20.err && \
timeout -k 10 200 python -m torch.distributed.run --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29513 bench.py --no-extras --no-cpu-baseline --allreduce --graph 0 > $O/ar_eager.json 2> $O/ar_eager.err
echo rc=$?

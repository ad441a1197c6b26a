set -o pipefail
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r4b
echo "== pmc faithful config 3 (sorted)" && PROF_SHAPE=config3 bash tools/gpu_pmc_faithful.sh r4b/pmcf3 sorted > gpurun_out/r4b/pmcf3.log 2>&1 \
 && python -c "import json; d=json.load(open('gpurun_out/r4b/pmcf3/pmc_faithful.json')); print(d['hbm_bytes_per_pass'])" \
&& echo "== pmc faithful config 2 (sorted)" && bash tools/gpu_pmc_faithful.sh r4b/pmcf2 sorted > gpurun_out/r4b/pmcf2.log 2>&1 \
 && python -c "import json; d=json.load(open('gpurun_out/r4b/pmcf2/pmc_faithful.json')); print(d['hbm_bytes_per_pass'])" \
&& echo "== gloo x2 rehearsal" && timeout -k 10 400 python bench.py --gpus 2 --backend gloo --steps 10 --warmup 2 --no-cpu-baseline \
  > gpurun_out/r4b/bench_gloo2.json 2> gpurun_out/r4b/bench_gloo2.err \
 && python -c "
import json; d=json.loads(open('gpurun_out/r4b/bench_gloo2.json').read().strip().splitlines()[-1])
print(d['value'], d['n_gpus'], json.dumps(d.get('collective')), json.dumps(d.get('faithful_sharded')), json.dumps(d.get('capi_group'))[:400])"

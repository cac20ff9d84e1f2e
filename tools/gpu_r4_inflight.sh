# HBM-origin probe (device-bound) at 64 vs 128 fragments in flight per player, interleaved,
# after the buffer-range decrypt:  bash tools/gpu_r4_inflight.sh -> gpurun_out/r4_inflight/*.log
set -eo pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/r4_inflight
mkdir -p $O
for i in 1 2; do
  for k in 64 128; do
    timeout -k 10 300 python bench.py --ingest hbm --inflight $k --steps 100 --warmup 6 > $O/hbm_k${k}_$i.log 2>&1
  done
done
for f in $O/*.log; do echo "$f $(grep -h '^{' $f | python3 -c 'import json,sys; j=json.loads(sys.stdin.readline()); print(j["value"], j["ms_per_step"], j["per_rank"][0]["bound"])')"; done

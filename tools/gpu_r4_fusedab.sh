# Fused receive verify vs the node's separate verify CRC (HLSP2P_DEFER_VERIFY=0) in the
# 2-rank HIP-IPC rehearsal with HBM origins, now that both ranks are transmux-bound
# (profiles/r4_soak run 2): 600 timed steps per run, 3 interleaved pairs.
#   bash tools/gpu_r4_fusedab.sh -> gpurun_out/r4_fusedab/*.log
set -eo pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/r4_fusedab
mkdir -p $O
reh() {  # $1 = HLSP2P_DEFER_VERIFY, $2 = port, rest: bench args
  HLSP2P_DEFER_VERIFY=$1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port $2 bench.py --gpus 2 --dist-backend ipc --ingest hbm --cache-gb 8 \
    --players 4 --verbose "${@:3}"
}
for i in 1 2 3; do
  reh 1 $((29970 + i)) --steps 600 --warmup 10 > $O/defer_$i.log 2>&1
  reh 0 $((29980 + i)) --steps 600 --warmup 10 > $O/node_$i.log 2>&1
done
for f in $O/*.log; do echo "$f $(grep -h '^{' $f | python3 -c 'import json,sys; j=json.loads(sys.stdin.readline()); print(j["value"], [(r["bound"], r["transmux_dev_ms"]) for r in j["per_rank"]])')"; done

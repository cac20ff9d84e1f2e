# 8 ranks sharing one MI355X over the HIP-IPC rehearsal plane: the N=8 code paths (7 peers
# per rank, 8-rank control messages and planner, IPC handles and event rings for 7 peers,
# deferred fused verify with corrupted copies) at small scale:
#   bash tools/gpu_r4_ipc8.sh -> gpurun_out/r4_ipc8/*.log
set -eo pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/r4_ipc8
mkdir -p $O
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
  --master-port 29961 bench.py --gpus 8 --dist-backend ipc --ingest hbm --cache-gb 2 --players 1 --inflight 16 \
  --steps 200 --warmup 10 --corrupt-recv 3 --verbose > $O/ipc8_hbm_corrupt.log 2>&1
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
  --master-port 29962 bench.py --gpus 8 --dist-backend ipc --cache-gb 2 --players 1 --inflight 16 \
  --steps 100 --warmup 5 --verbose > $O/ipc8_pcie.log 2>&1
for f in $O/*.log; do echo "== $f"; grep -h '^{' $f | python3 -c '
import json,sys
for l in sys.stdin:
    j=json.loads(l); print("value", j["value"], "ms", j["ms_per_step"], "offload", j.get("offload_ratio"))
    for r in j.get("per_rank", []): print("  rank", r.get("rank"), "cdn_GBps", r.get("cdn_GBps"), "p2p_GBps", r.get("p2p_GBps"), "crc_fail", r.get("crc_failures"), "bound", r.get("bound"))
'; done

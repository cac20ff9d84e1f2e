# 4 ranks on one MI355X over HIP IPC for 2,000 steps with HBM origins (3/4 of each rank's
# segments received and verified by the fused decrypt), 3 corrupted copies per rank:
#   bash tools/gpu_r4_ipc4soak.sh -> gpurun_out/r4_ipc4soak/*.log
set -eo pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/r4_ipc4soak
mkdir -p $O
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 \
  --master-port 29991 bench.py --gpus 4 --dist-backend ipc --ingest hbm --cache-gb 4 --players 2 --inflight 32 \
  --steps 2000 --warmup 10 --corrupt-recv 3 --verbose > $O/ipc4_hbm_2000.log 2>&1
grep -h '^{' $O/*.log | python3 -c '
import json,sys
for l in sys.stdin:
    j=json.loads(l); print("value", j["value"], "ms", j["ms_per_step"], "offload", j.get("offload_ratio"), "errors", j.get("errors"))
    for r in j.get("per_rank", []): print("  rank", r["rank"], "crc_fail", r["crc_failures"], "bound", r["bound"], "cdn_GBps", r["cdn_GBps"])
'

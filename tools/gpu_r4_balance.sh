# Planner CDN balance A/B on the one-GPU IPC rehearsal plane: per-rank cdn_GBps with the
# balance on (default) and off (HLSP2P_CDN_BALANCE=0), PCIe origin at 2 and 4 ranks, HBM at 2:
#   bash tools/gpu_r4_balance.sh  -> gpurun_out/r4_balance/*.log
set -eo pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/${BAL_OUT:-r4_balance}
mkdir -p $O
run() {  # name, nproc, port, balance, extra args...
  local name=$1 n=$2 port=$3 bal=$4; shift 4
  HLSP2P_CDN_BALANCE=$bal timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
    --master-addr 127.0.0.1 --master-port $port bench.py --gpus $n --dist-backend ipc --cache-gb 4 --players 2 \
    --inflight 32 --verbose "$@" > $O/$name.log 2>&1
}
run ipc2_pcie_on 2 29951 1 --steps 200 --warmup 10
run ipc2_pcie_off 2 29952 0 --steps 200 --warmup 10
run ipc4_pcie_on 4 29953 1 --steps 100 --warmup 5
run ipc4_pcie_off 4 29954 0 --steps 100 --warmup 5
run ipc2_hbm_on 2 29955 1 --ingest hbm --steps 300 --warmup 10
run ipc2_hbm_off 2 29956 0 --ingest hbm --steps 300 --warmup 10
for f in $O/*.log; do echo "== $f"; grep -h '^{' $f | python3 -c '
import json,sys
for l in sys.stdin:
    j=json.loads(l); print("value", j["value"], "ms", j["ms_per_step"])
    for r in j.get("per_rank", []): print("  rank", r.get("rank"), "cdn_GBps", r.get("cdn_GBps"), "bound", r.get("bound"), "xchg", r.get("exchange_GBps"))
'; done

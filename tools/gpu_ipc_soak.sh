# IPC rehearsal plane, default mode (host-side packing wait): short 2/4-rank runs and a
# 600-step 4-rank soak.
set -e
cd $GRAFT_REPO_ROOT
export PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/ipcsoak
mkdir -p $O
for N in 2 4; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 \
    --master-port $((29900 + N)) bench.py --gpus $N --steps 20 --warmup 4 --dist-backend ipc --cache-gb 4 \
    --players $((8 / N)) --verbose > $O/n${N}_pcie.log 2>&1
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 \
    --master-port $((29910 + N)) bench.py --gpus $N --steps 20 --warmup 4 --dist-backend ipc --cache-gb 4 \
    --players $((8 / N)) --ingest hbm --verbose > $O/n${N}_hbm.log 2>&1
done
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 \
  --master-port 29921 bench.py --gpus 4 --steps 600 --warmup 5 --dist-backend ipc --cache-gb 4 --players 2 \
  --verbose > $O/n4_soak600.log 2>&1

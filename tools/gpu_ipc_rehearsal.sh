# Multi-rank rehearsal on ONE MI355X with the device-to-device HIP-IPC data plane
# (bench.py --dist-backend ipc, parallel/comm.py:_IpcOutbox): the GPU test first, then
# 2- and 4-rank benches (PCIe origin and HBM-resident origin).
set -e
cd $GRAFT_REPO_ROOT
export PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/ipc
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_multirank_gpu.py -x -v --timeout 300 --timeout-method thread > $O/test.log 2>&1
for N in 2 4; do
  P=$((8 / N))
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 \
    --master-port $((29840 + N)) bench.py --gpus $N --steps 20 --warmup 4 --dist-backend ipc --cache-gb 4 \
    --players $P --verbose > $O/n${N}_pcie.log 2>&1
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 \
    --master-port $((29850 + N)) bench.py --gpus $N --steps 20 --warmup 4 --dist-backend ipc --cache-gb 4 \
    --players $P --ingest hbm --verbose > $O/n${N}_hbm.log 2>&1
done

# Multi-rank rehearsal on ONE MI355X (ranks share the GPU; RCCL cannot put two ranks on one
# device, so the data plane is gloo-staged or device-to-device HIP IPC):
#   bash tools/gpu_rehearsal.sh [ipc|gloo] [bench.py args ...]
#   -> the multi-rank GPU test, then 2- and 4-rank benches: gpurun_out/rehearsal/*.log
set -eo pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
PLANE=${1:-ipc}
shift || true
O=gpurun_out/rehearsal
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_multirank_gpu.py -x -v --timeout 300 --timeout-method thread > $O/test.log 2>&1
for N in 2 4; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 \
    --master-port $((29840 + N)) bench.py --gpus $N --steps 20 --warmup 4 --dist-backend $PLANE --cache-gb 4 \
    --players $((8 / N)) --verbose "$@" > $O/n${N}_${PLANE}.log 2>&1
  grep '^{' $O/n${N}_${PLANE}.log
done

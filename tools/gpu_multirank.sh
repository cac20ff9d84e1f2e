# Multi-rank rehearsal on ONE MI355X: N torchrun ranks share the GPU, gloo data plane
# (GPU tensors staged through host memory).  Exercises the whole N>1 bench path (control
# all-gather, planning, seeding + same-round forwarding, CRC trailers, async rounds,
# transmux) except RCCL itself, which cannot put two ranks on one GPU.
set -e
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out/multirank
for N in 2 4; do
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 \
    --master-port $((29600 + N)) bench.py --gpus $N --steps 10 --warmup 4 --dist-backend gloo --cache-gb 4 \
    --verbose > gpurun_out/multirank/n$N.log 2>&1
done

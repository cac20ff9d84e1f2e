# Rank-side cProfile of a 4-rank rehearsal on one GPU (gloo-staged data plane; the host
# phases of N>1 rounds -- plan, p2p layout, commit of received entries -- are what it
# measures).  Build the Cython modules with HLSP2P_CYTHON_PROFILE=1 beforehand.
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/mrprof
mkdir -p $O
HLSP2P_PROFILE=$O/n4 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
  --master-addr 127.0.0.1 --master-port 29834 bench.py --gpus 4 --steps 20 --warmup 3 --dist-backend gloo \
  --cache-gb 4 --players 2 --verbose > $O/n4.log 2>&1

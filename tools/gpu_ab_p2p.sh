# GPU tests, then a same-box A/B (ab_head = previous commit) of the P2P-phase host cost:
# 2- and 4-rank rehearsals on one GPU (gloo-staged data plane), host-cost config.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/abp2p
mkdir -p $O
cd $R
PYTHONPATH=$R timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
for N in 2 4; do
  for v in base new; do
    if [ $v = base ]; then cd $R/ab_head; else cd $R; fi
    PYTHONPATH=$PWD timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 \
      --master-port $((29700 + N + RANDOM % 50)) bench.py --gpus $N --steps 20 --warmup 5 --config hostcost --dist-backend gloo \
      --cache-gb 2 --verbose > $O/n${N}_${v}.log 2>&1
  done
done

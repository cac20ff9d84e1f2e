# Same-box A/B of the host path: ab_head/ (built copy of the previous commit) vs this tree,
# interleaved: 1-GPU host-cost probe x3 each, then a 2-rank rehearsal (gloo-staged data
# plane on one GPU) each for the P2P-phase bookkeeping.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/ab2
mkdir -p $O
for i in 1 2 3; do
  for v in base new; do
    if [ $v = base ]; then cd $R/ab_head; else cd $R; fi
    PYTHONPATH=$PWD timeout -k 10 200 python bench.py --config ${CONFIG:-hostcost} --steps 60 --warmup 10 --verbose > $O/h_${v}_$i.log 2>&1
  done
done
for v in base new; do
  if [ $v = base ]; then cd $R/ab_head; else cd $R; fi
  PYTHONPATH=$PWD timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port $((29650 + RANDOM % 100)) bench.py --gpus 2 --steps 20 --warmup 5 --config hostcost --dist-backend gloo \
    --cache-gb 2 --verbose > $O/n2_${v}.log 2>&1
done

# Fleet mode across configs and in multi-rank rehearsals (gloo-staged data plane on one GPU),
# plus a same-box single-process vs 2-player A/B of the host-bound probe.
set -e
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/fleet2
mkdir -p $O
for i in 1 2; do
  timeout -k 10 200 python bench.py --config hostcost --steps 40 --warmup 6 > $O/hc_p0_$i.log 2>&1
  timeout -k 10 200 python bench.py --config hostcost --steps 40 --warmup 6 --players 2 > $O/hc_p2_$i.log 2>&1
done
for c in abr5 4k25m 1080p6m-clear hostcost-abr; do
  timeout -k 10 200 python bench.py --config $c --players 2 --verbose > $O/$c.log 2>&1
done
for N in 2 4; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 \
    --master-port $((29820 + N)) bench.py --gpus $N --steps 10 --warmup 3 --dist-backend gloo --cache-gb 4 \
    --players 2 --verbose > $O/n$N.log 2>&1
done

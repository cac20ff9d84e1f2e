# Every bench config on the current tree (1 GPU) + 2/4-rank rehearsals on one GPU over the
# HIP-IPC data plane (incl. BASELINE config 3: ABR ladder under churn): catches native-path
# regressions outside the headline config.
set -e
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/cfg
mkdir -p $O
for c in 1080p6m 1080p6m-clear abr5 4k25m hostcost hostcost-abr; do
  timeout -k 10 200 python bench.py --config $c --verbose > $O/$c.log 2>&1
done
for N in 2 4; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 \
    --master-port $((29800 + N)) bench.py --gpus $N --steps 10 --warmup 3 --dist-backend ipc --cache-gb 4 \
    --players 2 --verbose > $O/n$N.log 2>&1
done
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29811 bench.py --gpus 2 --steps 20 --warmup 3 --dist-backend ipc --cache-gb 4 --config abr5 --churn 2 \
  --players 2 --verbose > $O/n2_abr5_churn.log 2>&1
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 \
  --master-port 29812 bench.py --gpus 4 --steps 20 --warmup 3 --dist-backend ipc --cache-gb 4 --config 4k25m \
  --players 2 --verbose > $O/n4_4k.log 2>&1

set -eo pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/r4_ipc8
mkdir -p $O
GPU_MAX_HW_QUEUES=2 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
  --master-port 29963 bench.py --gpus 8 --dist-backend ipc --ingest hbm --cache-gb 2 --players 1 --inflight 16 \
  --steps 200 --warmup 10 --corrupt-recv 3 --verbose > $O/ipc8_hbm_corrupt_q2.log 2>&1
GPU_MAX_HW_QUEUES=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
  --master-port 29964 bench.py --gpus 8 --dist-backend ipc --ingest hbm --cache-gb 2 --players 1 --inflight 16 \
  --steps 200 --warmup 10 --verbose > $O/ipc8_hbm_q1.log 2>&1

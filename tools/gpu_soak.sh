# Soak: long runs of the headline config and the rank-bound probe (the 8 GB HBM arena ring
# wraps ~100x), plus a long 4-rank IPC rehearsal.  Throughput must hold and peak memory
# must not grow with the step count (compare against the short runs).
set -e
cd $GRAFT_REPO_ROOT
export PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/soak
mkdir -p $O
timeout -k 10 200 python bench.py --steps 100 --warmup 5 --verbose > $O/headline_100.log 2>&1
timeout -k 10 400 python bench.py --steps 2000 --warmup 5 --verbose > $O/headline_2000.log 2>&1
timeout -k 10 200 python bench.py --ingest hbm --steps 100 --warmup 5 --verbose > $O/hbm_100.log 2>&1
timeout -k 10 400 python bench.py --ingest hbm --steps 4000 --warmup 5 --verbose > $O/hbm_4000.log 2>&1
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 \
  --master-port 29891 bench.py --gpus 4 --steps 600 --warmup 5 --dist-backend ipc --cache-gb 4 --players 2 \
  --verbose > $O/n4_ipc_600.log 2>&1

set -e
cd $GRAFT_REPO_ROOT
export PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/ipc2
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_multirank_gpu.py -x -v --timeout 300 --timeout-method thread > $O/test.log 2>&1
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 \
    --master-port 29864 bench.py --gpus 4 --steps 20 --warmup 4 --dist-backend ipc --cache-gb 4 \
    --players 2 --ingest hbm --verbose > $O/n4_hbm.log 2>&1

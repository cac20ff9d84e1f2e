# GPU tests + multi-rank rehearsal (gloo data plane, N=2/4 on one GPU) + 1-GPU headline bench.
set -e
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
mkdir -p gpurun_out/check
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/check/gpu_tests.log 2>&1
for N in 2 4; do
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 \
    --master-port $((29600 + N)) bench.py --gpus $N --steps 10 --warmup 4 --dist-backend gloo --cache-gb 4 \
    --verbose > gpurun_out/check/n$N.log 2>&1
done
timeout -k 10 300 python bench.py --verbose > gpurun_out/check/bench_1080p.log 2>&1

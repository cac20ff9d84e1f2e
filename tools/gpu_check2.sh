set -e
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
mkdir -p gpurun_out/check2
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/check2/gpu_tests.log 2>&1
for N in 2 4; do
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 \
    --master-port $((29600 + N)) bench.py --gpus $N --steps 10 --warmup 4 --dist-backend gloo --cache-gb 4 \
    --verbose > gpurun_out/check2/n$N.log 2>&1
done
for c in hostcost 4k25m abr5; do
  timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 6 --verbose > gpurun_out/check2/$c.log 2>&1
done
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/check2/smoke.log 2>&1

# Validation with the fleet default: GPU tests, smoke, headline bench (default = 4 players)
# and single-process, host-bound probe, 2/4-rank rehearsals (HIP-IPC data plane; the gloo-staged
# plane is covered by tests/test_multirank_gpu.py).
set -e
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/vfleet
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 300 python bench.py > $O/bench_default_1.log 2>&1
timeout -k 10 300 python bench.py --players 0 > $O/bench_p0.log 2>&1
timeout -k 10 300 python bench.py > $O/bench_default_2.log 2>&1
timeout -k 10 300 python bench.py --config hostcost --steps 40 --warmup 6 --verbose > $O/hostcost_default.log 2>&1
timeout -k 10 300 python bench.py --ingest hbm --steps 30 --warmup 5 --verbose > $O/hbm_default.log 2>&1
for N in 2 4; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 \
    --master-port $((29830 + N)) bench.py --gpus $N --steps 10 --warmup 3 --dist-backend ipc --cache-gb 4 --players 2 \
    --verbose > $O/n$N.log 2>&1
done

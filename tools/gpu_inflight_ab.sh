set -e
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
mkdir -p gpurun_out/kab
for i in 1 2; do
  for K in 64 128 256; do
    timeout -k 10 200 python bench.py --config hostcost --inflight $K --steps 20 --warmup 6 --verbose > gpurun_out/kab/hc_k${K}_$i.log 2>&1
  done
done
for K in 64 128; do
  timeout -k 10 200 python bench.py --inflight $K --steps 20 --warmup 6 --verbose > gpurun_out/kab/1080_k${K}.log 2>&1
done

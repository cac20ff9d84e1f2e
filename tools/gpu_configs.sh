# The bench's other BASELINE configs on one GPU (ABR ladder, 4K, clear, cache saturation)
set -e
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out/configs
for c in ${CONFIGS:-abr5 4k25m 1080p6m-clear}; do
  timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 6 --verbose > gpurun_out/configs/$c.log 2>&1
done
# 4K with a 2 GB arena: the ring is smaller than 3 rounds in flight -> backpressure
timeout -k 10 300 python bench.py --config 4k25m --cache-gb 2 --steps 20 --warmup 6 --verbose > gpurun_out/configs/4k25m_cache2g.log 2>&1
HLSP2P_PROFILE=gpurun_out/configs/pabr5 timeout -k 10 300 python bench.py --config abr5 --steps 20 --warmup 6 > gpurun_out/configs/abr5_prof.log 2>&1

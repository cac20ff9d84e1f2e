set -o pipefail
mkdir -p gpurun_out/r2b
HLSJS_P2P_PURE=1 HLSP2P_PROFILE=gpurun_out/r2b/prof_pure timeout -k 10 180 python bench.py --config hostcost --steps 60 --warmup 10 --verbose > gpurun_out/r2b/hostcost_pure.log 2>&1 &&
for i in 1 2 3; do timeout -k 10 120 python bench.py --config hostcost --steps 60 --warmup 10 > gpurun_out/r2b/hostcost_$i.log 2>&1 || exit 1; done

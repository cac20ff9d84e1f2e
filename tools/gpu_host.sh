# Host-overhead analysis on the GPU box: cProfile of the timed steps (1080p and the tiny
# "hostcost" config where per-segment Python cost dominates).
set -e
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out/host
HLSP2P_PROFILE=gpurun_out/host/p1080 timeout -k 10 300 python bench.py --steps 20 --warmup 6 --verbose > gpurun_out/host/b1080.log 2>&1
HLSP2P_PROFILE=gpurun_out/host/phc timeout -k 10 300 python bench.py --steps 20 --warmup 6 --verbose --config hostcost > gpurun_out/host/bhc.log 2>&1
timeout -k 10 300 python bench.py --steps 20 --warmup 6 --verbose > gpurun_out/host/b1080_noprof.log 2>&1
timeout -k 10 300 python bench.py --steps 20 --warmup 6 --verbose --config hostcost > gpurun_out/host/bhc_noprof.log 2>&1

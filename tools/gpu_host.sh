# Host-path profile on one MI355X: the 1080p bench with the Cython-compiled hot path and in
# pure-Python mode under cProfile (per-function host cost per segment), plus the
# 30 KB-segment host-ceiling probe.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/host
timeout -k 10 300 python bench.py --steps 30 --warmup 6 --verbose > gpurun_out/host/bench_1080p.log 2>&1
timeout -k 10 300 python bench.py --config hostcost --steps 30 --warmup 6 --verbose > gpurun_out/host/bench_hostcost.log 2>&1
HLSJS_P2P_PURE=1 HLSP2P_PROFILE=gpurun_out/host/cprofile_pure timeout -k 10 300 python bench.py --config hostcost --steps 30 --warmup 6 --verbose > gpurun_out/host/bench_hostcost_pure_prof.log 2>&1

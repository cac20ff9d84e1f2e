# Host-path profile with the Cython modules built with profile=True (HLSP2P_CYTHON_PROFILE=1
# build beforehand): cProfile sees the compiled functions, so the per-function split is the
# one of the compiled hot path (absolute times inflated by the profiling hooks).
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/cyprof
HLSP2P_PROFILE=gpurun_out/cyprof/hostcost timeout -k 10 300 python bench.py --config hostcost --steps 60 --warmup 6 --verbose > gpurun_out/cyprof/hostcost.log 2>&1
timeout -k 10 300 python bench.py --config hostcost --steps 60 --warmup 6 > gpurun_out/cyprof/hostcost_noprof.log 2>&1

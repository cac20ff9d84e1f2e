# Rank-side cProfile of the fleet (4 players) on the HBM-ingest probe; run with the Cython
# modules built with HLSP2P_CYTHON_PROFILE=1 so cProfile sees the compiled functions.
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/fleetprof
mkdir -p $O
HLSP2P_PROFILE=$O/hbm timeout -k 10 300 python bench.py --ingest hbm --steps 60 --warmup 6 --verbose > $O/hbm.log 2>&1
HLSP2P_PROFILE=$O/hostcost timeout -k 10 300 python bench.py --config hostcost --steps 60 --warmup 6 --verbose > $O/hostcost.log 2>&1

# HBM-origin probe: kernel time per step (rocprofv3 kernel trace) and the player count
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r3b
timeout -k 10 300 python bench.py --steps 100 --warmup 10 --ingest hbm --players 6 --verbose > $R/gpurun_out/r3b/hbm_p6.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 100 --warmup 10 --config hostcost --players 6 --verbose > $R/gpurun_out/r3b/hostcost_p6.log 2>&1 &&
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $R/gpurun_out/r3b/prof -o run --output-format csv -- python $R/bench.py --steps 50 --warmup 10 --ingest hbm > $R/gpurun_out/r3b/prof.log 2>&1

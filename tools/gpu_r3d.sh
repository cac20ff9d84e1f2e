# fused decrypt + demux: GPU suite, probes (fused vs split, same box), headline, kernel profile
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r3d
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $R/gpurun_out/r3d/gpu_tests.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 100 --warmup 10 --ingest hbm --players 6 --verbose > $R/gpurun_out/r3d/hbm_p6.log 2>&1 &&
HLSP2P_TRANSMUX=split timeout -k 10 300 python bench.py --steps 100 --warmup 10 --ingest hbm --players 6 --verbose > $R/gpurun_out/r3d/hbm_p6_split.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 100 --warmup 10 --ingest hbm --players 6 --verbose > $R/gpurun_out/r3d/hbm_p6_b.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $R/gpurun_out/r3d/bench.log 2>&1 &&
timeout -k 10 300 python bench.py --config 1080p6m-live --steps 400 --warmup 20 --players 4 --verbose > $R/gpurun_out/r3d/live.log 2>&1 &&
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r3d/prof -o run --output-format csv -- python $R/bench.py --steps 50 --warmup 10 --ingest hbm --players 6 > $R/gpurun_out/r3d/prof.log 2>&1

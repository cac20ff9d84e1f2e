# kernel-level trace of one isolated transmux batch, split vs fused (rocprofv3 --stats)
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r3g
cd /tmp && export TMPDIR=/tmp
PYTHONPATH=$R timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r3g/prof -o run -- python3 $R/tools/transmux_bench.py --segs 256 --iters 10 > $R/gpurun_out/r3g/tb.log 2>&1

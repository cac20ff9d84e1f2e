# RCCL progress under a concurrent decrypt batch (one-rank native RCCL self-exchange on one
# stream, a 3 MB-segment transmux batch on another), for several CU reserves and RCCL CTA
# caps; then a kernel trace of the concurrent case.
#   bash tools/gpu_rccl_overlap.sh [trace]   -> gpurun_out/rccl_overlap/*
set -eo pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/rccl_overlap
mkdir -p $O
cd $R
ov() { PYTHONPATH=$R timeout -k 10 200 python tools/rccl_overlap.py --segs 128 --msgs 64 "$@"; }
ov --reserves 0,8,16 > $O/default.log 2>&1
NCCL_MIN_CTAS=8 NCCL_MAX_CTAS=8 ov --reserves 8,16 > $O/ctas8.log 2>&1
NCCL_MIN_CTAS=16 NCCL_MAX_CTAS=16 ov --reserves 16,32 > $O/ctas16.log 2>&1
NCCL_MIN_CTAS=4 NCCL_MAX_CTAS=4 ov --reserves 4,8 > $O/ctas4.log 2>&1
grep -h '^{' $O/default.log $O/ctas8.log $O/ctas16.log $O/ctas4.log
if [ "${1:-}" = trace ]; then
  cd /tmp && export TMPDIR=/tmp
  NCCL_MIN_CTAS=8 NCCL_MAX_CTAS=8 PYTHONPATH=$R timeout -k 10 300 rocprofv3 --kernel-trace -d $O/db -o run -- python3 $R/tools/rccl_overlap.py --segs 128 --msgs 64 --reserves 8 --iters 2 > $O/prof.log 2>&1
  python3 $R/tools/rocpd_kernels.py $(ls $O/db/*.db | head -1) --timeline 60 > $O/kernels_ctas8.txt
fi

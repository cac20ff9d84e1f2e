# The N=8 driver shape at bench defaults (4 players x 64 in flight per rank) over the native
# RCCL plane, 8 ranks sharing ONE MI355X (socket transport rehearsal; GPU_MAX_HW_QUEUES=1).
set -eo pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R HLSP2P_RCCL_REHEARSAL=socket GPU_MAX_HW_QUEUES=1
O=gpurun_out/r5_rccl
mkdir -p $O
timeout -k 10 900 python -u bench.py --gpus 8 --steps 6 --warmup 2 --cache-gb 4 > $O/n8_full.log 2>&1
grep -h '^{' $O/n8_full.log | cut -c1-300

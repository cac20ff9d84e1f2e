# The native RCCL plane at bench scale with 2 ranks sharing the GPU (socket transport):
# 4 players x 64 in flight per rank, 6 GB arenas, 150 timed rounds (ring wraps, entry ids
# past 1024, the divergence check every round).
set -eo pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R HLSP2P_RCCL_REHEARSAL=socket
O=gpurun_out/r5_rccl
mkdir -p $O
timeout -k 10 600 python -u bench.py --gpus 2 --steps 150 --warmup 5 --cache-gb 6 --verbose > $O/n2_scale.log 2>&1
grep -h '^{' $O/n2_scale.log | cut -c1-300

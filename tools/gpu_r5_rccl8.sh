# Native RCCL plane at N=8 on ONE MI355X over RCCL's socket transport (rehearsal), plus the
# new GPU test.  GPU_MAX_HW_QUEUES=1: eight processes on one GPU otherwise time-slice its
# hardware queues (profiles/r4_ipc8).
set -eo pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/r5_rccl
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_multirank_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread -k sharing_the_gpu > $O/test.log 2>&1
HLSP2P_RCCL_REHEARSAL=socket GPU_MAX_HW_QUEUES=1 timeout -k 10 500 python -u bench.py --gpus 8 --steps 10 --warmup 3 --cache-gb 2 --inflight 16 --players 1 --corrupt-recv 3 > $O/n8_corrupt.log 2>&1
tail -3 $O/test.log
grep -h '^{' $O/n8_corrupt.log | cut -c1-400

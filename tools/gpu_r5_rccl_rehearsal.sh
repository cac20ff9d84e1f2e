# The native RCCL data plane with several ranks on ONE MI355X: each rank presents its own
# NCCL_HOSTID, so RCCL connects them over its socket transport instead of refusing duplicate
# devices (parallel/comm.py HLSP2P_RCCL_REHEARSAL=socket).  bench.py self-launches the ranks.
set -eo pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R HLSP2P_RCCL_REHEARSAL=socket NCCL_DEBUG=WARN
O=gpurun_out/r5_rccl
mkdir -p $O
timeout -k 10 300 python -u bench.py --gpus 2 --steps 10 --warmup 3 --cache-gb 2 --inflight 16 --players 2 --verbose > $O/n2.log 2>&1
grep -h '^{' $O/n2.log | cut -c1-600
timeout -k 10 300 python -u bench.py --gpus 2 --steps 10 --warmup 3 --cache-gb 2 --inflight 16 --players 0 --corrupt-recv 3 --ingest hbm > $O/n2_corrupt_p0.log 2>&1
timeout -k 10 300 python -u bench.py --gpus 4 --steps 10 --warmup 3 --cache-gb 2 --inflight 16 --players 1 --corrupt-recv 3 > $O/n4_corrupt.log 2>&1
grep -h '^{' $O/n2_corrupt_p0.log $O/n4_corrupt.log | cut -c1-400

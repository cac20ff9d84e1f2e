# Third batch of native-RCCL-plane stress cases (ranks sharing ONE MI355X over the socket
# transport): fleet payloads at N=2, 128 in flight per player at N=8, and the host-cost
# config (many small segments) at N=8.  The first failure ends it.
set -eo pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R HLSP2P_RCCL_REHEARSAL=socket GPU_MAX_HW_QUEUES=1
O=gpurun_out/r5_rccl_stress3
mkdir -p $O
timeout -k 10 400 python -u bench.py --gpus 2 --fleet-payload --steps 150 --warmup 5 > $O/n2_payload.log 2>&1
timeout -k 10 400 python -u bench.py --gpus 8 --inflight 128 --steps 20 --warmup 3 --cache-gb 6 > $O/n8_inflight128.log 2>&1
timeout -k 10 400 python -u bench.py --gpus 8 --config hostcost --steps 100 --warmup 5 --cache-gb 2 > $O/n8_hostcost.log 2>&1
grep -h '^{' $O/*.log | cut -c1-200

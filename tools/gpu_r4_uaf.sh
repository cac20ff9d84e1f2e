# Round 4: the CRC-table stream-lifetime fix (agent/node.py ownership rule), on one MI355X:
#   bash tools/gpu_r4_uaf.sh   -> gpurun_out/r4_uaf/*.log
#   1. the stream-safety GPU tests (positive control of the race + the node's grow path)
#   2. the round-3 faulting rehearsal, unchanged: 2 ranks on one GPU, HIP-IPC data plane with
#      interprocess events, 128 fragments in flight per player, 4 players, 12 GB arena
set -eo pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/r4_uaf
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_stream_safety_gpu.py -x -v --timeout 120 --timeout-method thread > $O/stream_tests.log 2>&1
HLSP2P_IPC_EVENTS=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29851 bench.py --gpus 2 --steps 60 --warmup 4 --dist-backend ipc \
  --cache-gb 12 --players 4 --inflight 128 --verbose > $O/n2_ipc_inflight128_events.log 2>&1
grep '^{' $O/n2_ipc_inflight128_events.log
timeout -k 10 700 python -u -m pytest tests/test_multirank_gpu.py -x -v --timeout 650 --timeout-method thread > $O/multirank_tests.log 2>&1

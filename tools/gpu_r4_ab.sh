# Round 4 A/B runs on one MI355X:  bash tools/gpu_r4_ab.sh  -> gpurun_out/r4_ab/*.log
#   * the stream-safety GPU tests (positive control + the node's grow path)
#   * headline at 64 vs 128 fragments in flight per player (interleaved, 2 runs each) and the
#     HBM-origin probe at both (the default in-flight count is chosen from these)
#   * headline with fleet payloads (every player's onSuccess carries the bytes)
#   * the replicated planner's host cost on this box's CPU (tools/planner_cost.py)
#   * which IPC exports each HSA IPC mode allows (tools/ipc_mode_probe.py)
set -eo pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/r4_ab
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_stream_safety_gpu.py tests/test_transmux.py tests/test_kernels_gpu.py tests/test_torch_ops.py -v --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 300 python tools/transmux_bench.py --segs 256 --iters 10 > $O/transmux_bench.log 2>&1
for i in 1 2; do
  timeout -k 10 300 python bench.py --inflight 64 --verbose > $O/head64_$i.log 2>&1
  timeout -k 10 300 python bench.py --inflight 128 --verbose > $O/head128_$i.log 2>&1
done
timeout -k 10 300 python bench.py --ingest hbm --steps 100 --warmup 6 --inflight 64 --verbose > $O/hbm64.log 2>&1
timeout -k 10 300 python bench.py --ingest hbm --steps 100 --warmup 6 --inflight 128 --verbose > $O/hbm128.log 2>&1
timeout -k 10 300 python bench.py --fleet-payload --verbose > $O/head_payload.log 2>&1
timeout -k 10 300 python bench.py --fleet-payload --ingest hbm --steps 100 --warmup 6 --verbose > $O/hbm_payload.log 2>&1
timeout -k 10 300 python tools/planner_cost.py --world 2 8 --wants 256 512 1024 > $O/planner_cost.log 2>&1
HSA_ENABLE_IPC_MODE_LEGACY=0 timeout -k 10 120 python tools/ipc_mode_probe.py > $O/ipc_mode0.log 2>&1
HSA_ENABLE_IPC_MODE_LEGACY=1 timeout -k 10 120 python tools/ipc_mode_probe.py > $O/ipc_mode1.log 2>&1
grep -h '^{' $O/*.log | cut -c1-400

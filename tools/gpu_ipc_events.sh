# Root-cause probe of the HIP interprocess-event failure (parallel/comm.py _IpcOutbox,
# HLSP2P_IPC_EVENTS=1): the protocol's event traffic alone, N ranks on one GPU, several modes.
#   bash tools/gpu_ipc_events.sh   -> gpurun_out/ipc_events/*.log
set -eo pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/ipc_events
mkdir -p $O
run() { timeout -k 10 150 python -m torch.distributed.run --nnodes=1 --nproc-per-node $1 --master-addr 127.0.0.1 --master-port $2 tools/ipc_event_probe.py "${@:3}"; }
run 2 29611 --mode wait --rounds 2000 > $O/wait_n2.log 2>&1
run 4 29612 --mode wait --rounds 1500 > $O/wait_n4.log 2>&1
run 4 29613 --mode wait --rounds 1500 --send-prob 0.6 > $O/wait_n4_sparse.log 2>&1
run 4 29614 --mode query --rounds 1500 > $O/query_n4.log 2>&1
run 4 29615 --mode reopen --rounds 1500 --every 50 > $O/reopen_n4.log 2>&1
grep -h -A4 "mode=" $O/*.log

# HIP interprocess events on the one-GPU rehearsal plane (parallel/comm.py _IpcOutbox):
#   bash tools/gpu_ipc_events.sh probe   the protocol's event traffic alone, N ranks, several modes
#                                        (root cause: an IPC event survives 32 records)
#   bash tools/gpu_ipc_events.sh soak    4-rank 600-step rehearsal bench, event mode vs host waits
#   -> gpurun_out/ipc_events/*.log
set -eo pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/ipc_events
mkdir -p $O
run() { timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node $1 --master-addr 127.0.0.1 --master-port $2 tools/ipc_event_probe.py "${@:3}"; }
soak() {  # $1 = HLSP2P_IPC_EVENTS, $2 = port
  HLSP2P_IPC_EVENTS=$1 timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 \
    --master-port $2 bench.py --gpus 4 --steps 600 --warmup 5 --dist-backend ipc --cache-gb 4 --players 2 --verbose
}
case ${1:-probe} in
  probe)
    run 2 29611 --mode wait --rounds 2000 > $O/wait_n2.log 2>&1
    run 4 29612 --mode wait --rounds 1500 > $O/wait_n4.log 2>&1
    run 4 29613 --mode wait --rounds 1500 --send-prob 0.6 > $O/wait_n4_sparse.log 2>&1
    run 4 29614 --mode query --rounds 1500 > $O/query_n4.log 2>&1
    run 4 29615 --mode reopen --rounds 1500 --every 20 > $O/reopen_n4.log 2>&1
    run 4 29616 --mode renew --rounds 3000 > $O/renew_n4.log 2>&1
    run 4 29617 --mode renew --rounds 3000 --send-prob 0.6 > $O/renew_n4_sparse.log 2>&1
    grep -h -A4 "mode=" $O/*.log ;;
  soak)
    soak 1 29621 > $O/soak_n4_events.log 2>&1
    soak 0 29622 > $O/soak_n4_hostwait.log 2>&1
    grep -h '^{' $O/soak_n4_events.log $O/soak_n4_hostwait.log ;;
esac

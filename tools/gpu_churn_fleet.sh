# BASELINE config 3 (5-rendition ABR ladder under swarm churn) with the fleet default on one
# GPU over the HIP-IPC rehearsal plane: calm vs --churn 2, 2 and 4 ranks.
set -e
cd $GRAFT_REPO_ROOT
export PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/churn
mkdir -p $O
for N in 2 4; do
  for C in 0 2; do
    timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 \
      --master-port $((29870 + N * 3 + C)) bench.py --gpus $N --steps 24 --warmup 3 --dist-backend ipc --cache-gb 4 \
      --config abr5 --churn $C --players 2 --verbose > $O/n${N}_churn$C.log 2>&1
  done
done

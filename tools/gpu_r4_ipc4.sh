# 4 ranks sharing one MI355X over the HIP-IPC rehearsal plane (the N>2 code paths: 3 peers per
# rank, seeding quotas, deferred fused verify with several sources, corrupted copies):
#   bash tools/gpu_r4_ipc4.sh  -> gpurun_out/r4_ipc4/*.log
set -eo pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/r4_ipc4
mkdir -p $O
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 \
  --master-port 29941 bench.py --gpus 4 --dist-backend ipc --ingest hbm --cache-gb 4 --players 2 --inflight 32 \
  --steps 300 --warmup 10 --corrupt-recv 3 --verbose > $O/ipc4_hbm_corrupt.log 2>&1
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 \
  --master-port 29942 bench.py --gpus 4 --dist-backend ipc --cache-gb 4 --players 2 --inflight 32 \
  --steps 100 --warmup 5 --verbose > $O/ipc4_pcie.log 2>&1
grep -h '^{' $O/*.log | cut -c1-260

# Round-4 soak on one MI355X: the headline for 2,000 steps, and the 2-rank HIP-IPC rehearsal
# with HBM origins (half of each rank's segments received, fused-verify path) for 3,000 steps.
#   bash tools/gpu_r4_soak.sh  -> gpurun_out/r4_soak/*.log
set -eo pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/${SOAK_OUT:-r4_soak}
mkdir -p $O
timeout -k 10 300 python bench.py --steps 2000 --warmup 10 --verbose > $O/headline_2000.log 2>&1
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29931 bench.py --gpus 2 --dist-backend ipc --ingest hbm --cache-gb 8 --players 4 \
  --steps 3000 --warmup 10 --verbose > $O/ipc2_hbm_3000.log 2>&1
grep -h '^{' $O/*.log | cut -c1-300

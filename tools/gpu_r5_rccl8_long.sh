# Longer N=8 / N=4 runs of the native RCCL plane at the bench defaults (4 players x 64 in
# flight per rank), ranks sharing ONE MI355X over RCCL's socket transport, with injected
# transport corruption; the final round-5 tree, self-launched (bench.py --gpus N).
set -eo pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R HLSP2P_RCCL_REHEARSAL=socket GPU_MAX_HW_QUEUES=1
O=gpurun_out/r5_rccl_long
mkdir -p $O
timeout -k 10 500 python -u bench.py --gpus 8 --steps 60 --warmup 3 --cache-gb 4 --corrupt-recv 5 > $O/n8_long.log 2>&1
timeout -k 10 400 python -u bench.py --gpus 4 --steps 120 --warmup 3 --cache-gb 6 > $O/n4_long.log 2>&1
grep -h '^{' $O/*.log | cut -c1-300

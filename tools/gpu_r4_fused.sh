# Round 4: the receive-side CRC fused into the decrypt, A/B on one MI355X.
#   bash tools/gpu_r4_fused.sh   -> gpurun_out/r4_fused/*.log
#   * 2-rank HIP-IPC rehearsal with HBM origins (every rank receives half its segments from the
#     other): deferred verify (the CRC fused into the transmux's decrypt) vs the node's separate
#     verify CRC (HLSP2P_DEFER_VERIFY=0), interleaved, 2 runs each
#   * the same with a corrupted peer copy in each of the first 3 timed rounds (caught, re-fetched)
#   * kernel trace of one deferred-verify rehearsal (per-kernel time per segment)
set -eo pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/${FUSED_OUT:-r4_fused}
mkdir -p $O
reh() {  # $1 = HLSP2P_DEFER_VERIFY, $2 = port, rest: bench args
  HLSP2P_DEFER_VERIFY=$1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port $2 bench.py --gpus 2 --dist-backend ipc --ingest hbm --cache-gb 8 \
    --players 4 --verbose "${@:3}"
}
for i in 1 2; do
  reh 1 $((29900 + i)) --steps 60 --warmup 6 > $O/defer_$i.log 2>&1
  reh 0 $((29910 + i)) --steps 60 --warmup 6 > $O/node_$i.log 2>&1
done
reh 1 29921 --steps 30 --warmup 6 --corrupt-recv 3 > $O/defer_corrupt.log 2>&1
grep -h '^{' $O/*.log | cut -c1-300
timeout -k 10 300 python tools/transmux_bench.py --segs 256 --iters 10 --verify > $O/transmux_verify.log 2>&1
cd /tmp && export TMPDIR=/tmp
PYTHONPATH=$R timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o run -- python3 $R/tools/transmux_bench.py --segs 256 --iters 5 --verify > $R/$O/prof.log 2>&1
cat $R/$O/transmux_verify.log

# Fleet round size: fragments per player and round (--inflight) on the rank-bound probe
# (HBM-resident origin, 1080p AES), interleaved passes.
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/inflight_fleet
mkdir -p $O
for rep in 1 2 3; do
  for k in 64 128 192; do
    timeout -k 10 200 python bench.py --ingest hbm --inflight $k --steps 30 --warmup 5 --verbose > $O/hbm_k${k}_$rep.log 2>&1
  done
done

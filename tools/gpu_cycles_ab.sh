# Soak A/B: break the fleet's Pending<->Request reference cycle at completion (1) or leave it
# to the cyclic GC (0); HBM-resident origin probe, 4000 steps, interleaved.
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/cycles
mkdir -p $O
for rep in 1 2; do
  for v in 0 1; do
    HLSP2P_BREAK_CYCLES=$v timeout -k 10 300 python bench.py --ingest hbm --steps 4000 --warmup 5 --verbose > $O/hbm4000_b${v}_$rep.log 2>&1
  done
done
timeout -k 10 200 python bench.py --ingest hbm --steps 100 --warmup 5 --verbose > $O/hbm100_b1.log 2>&1

# Long-run diagnostic: HBM-origin fleet probe over 3000 steps with the cyclic GC on (default
# tuning) and fully disabled after start-up, plus a 100-step reference; peak host memory shows
# what the GC would have reclaimed.
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/gcab
mkdir -p $O
timeout -k 10 200 python bench.py --ingest hbm --steps 100 --warmup 5 --verbose > $O/s100.log 2>&1
for rep in 1 2; do
  timeout -k 10 300 python bench.py --ingest hbm --steps 3000 --warmup 5 --verbose > $O/s3000_gc_$rep.log 2>&1
  HLSP2P_GC_DISABLE=1 timeout -k 10 300 python bench.py --ingest hbm --steps 3000 --warmup 5 --verbose > $O/s3000_nogc_$rep.log 2>&1
done

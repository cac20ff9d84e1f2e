# Long-run A/B of the GC tuning: full collections 10x rarer (new default) vs GC disabled after
# start-up, HBM-origin fleet probe over 3000 steps, interleaved; plus the 100-step reference.
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/gcab2
mkdir -p $O
timeout -k 10 200 python bench.py --ingest hbm --steps 100 --warmup 5 --verbose > $O/s100.log 2>&1
for rep in 1 2; do
  timeout -k 10 300 python bench.py --ingest hbm --steps 3000 --warmup 5 --verbose > $O/s3000_gc_$rep.log 2>&1
  HLSP2P_GC_DISABLE=1 timeout -k 10 300 python bench.py --ingest hbm --steps 3000 --warmup 5 --verbose > $O/s3000_nogc_$rep.log 2>&1
done
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $O/headline.log 2>&1

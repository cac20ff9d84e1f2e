# Same-box A/B: ab_head (HEAD) vs this tree on the rank-bound probes (HBM-ingest 1080p and
# hostcost), x5 pairs alternating which variant runs first.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/abcols
mkdir -p $O
for i in 1 2 3 4 5; do
  if [ $((i % 2)) = 1 ]; then order="base new"; else order="new base"; fi
  for v in $order; do
    if [ $v = base ]; then cd $R/ab_head; else cd $R; fi
    PYTHONPATH=$PWD timeout -k 10 200 python bench.py --ingest hbm --steps 30 --warmup 5 --verbose > $O/hbm_${v}_$i.log 2>&1
    PYTHONPATH=$PWD timeout -k 10 200 python bench.py --config hostcost --steps 40 --warmup 6 --verbose > $O/hc_${v}_$i.log 2>&1
  done
done

# A/B of the host path on ONE box: baseline tree (ab_base/, an older commit, built) vs this
# tree, alternated so box-to-box CPU variance cancels.
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/ab
for i in 1 2; do
  for v in base new; do
    if [ $v = base ]; then cd $R/ab_base; else cd $R; fi
    timeout -k 10 200 python bench.py --config hostcost --steps 30 --warmup 6 --verbose > $R/gpurun_out/ab/hostcost_${v}_$i.log 2>&1
    timeout -k 10 200 python bench.py --steps 30 --warmup 6 --verbose > $R/gpurun_out/ab/1080p_${v}_$i.log 2>&1
  done
done

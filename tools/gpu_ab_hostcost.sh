# Interleaved A/B of the host-cost probe: the tree in _ab/ (A) against this tree (B).
set -eo pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/ab_hostcost
mkdir -p $O
for i in 1 2 3; do
  (cd $R/_ab && PYTHONPATH=$R/_ab timeout -k 10 200 python bench.py --config hostcost --steps 300 --warmup 20 > $O/A$i.log 2>&1)
  (cd $R && PYTHONPATH=$R timeout -k 10 200 python bench.py --config hostcost --steps 300 --warmup 20 > $O/B$i.log 2>&1)
done
for f in $O/A*.log $O/B*.log; do echo "$(basename $f) $(grep -h '^{' $f | cut -c90-115)"; done

# Same-box A/B of the host path: ab_head/ (a built copy of the previous commit) vs this tree,
# interleaved so box-to-box CPU variance cancels.  Args: bench config(s), default hostcost.
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/abtree
for i in 1 2 3; do
  for v in base new; do
    if [ $v = base ]; then cd $R/ab_head; else cd $R; fi
    for c in ${CONFIGS:-hostcost}; do
      PYTHONPATH=$PWD timeout -k 10 200 python bench.py --config $c --steps 30 --warmup 6 --verbose > $R/gpurun_out/abtree/${c}_${v}_$i.log 2>&1
    done
  done
done

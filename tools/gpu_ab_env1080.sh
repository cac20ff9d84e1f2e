# Same-box A/B of an env switch on the 1-GPU headline: VAR=A vs VAR=B, interleaved x3.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/abenv1080
mkdir -p $O
cd $R
for i in 1 2 3; do
  for v in $2 $3; do
    env $1=$v PYTHONPATH=$R timeout -k 10 200 python bench.py --verbose > $O/${1}_${v}_$i.log 2>&1
  done
done

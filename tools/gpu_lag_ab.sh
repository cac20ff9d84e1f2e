# Same-box A/B of the bench's round lag (1 = the previous pipeline, 2 = default), interleaved.
set -e
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
mkdir -p gpurun_out/lag
for i in 1 2 3; do
  for L in 1 2; do
    timeout -k 10 200 python bench.py --verbose --lag $L "$@" > gpurun_out/lag/lag${L}_$i.log 2>&1
  done
done

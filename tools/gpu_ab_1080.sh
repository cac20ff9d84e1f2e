# Same-box A/B of the 1-GPU headline (1080p AES): ab_head vs this tree, interleaved x3.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/ab1080
mkdir -p $O
for i in 1 2 3; do
  for v in base new; do
    if [ $v = base ]; then cd $R/ab_head; else cd $R; fi
    PYTHONPATH=$PWD timeout -k 10 200 python bench.py --verbose > $O/${v}_$i.log 2>&1
  done
done

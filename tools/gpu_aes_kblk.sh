# AES chains per lane: kBlk=4 (this tree) vs kBlk=5 (ab_head), kernel bench interleaved x3.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/aeskb
mkdir -p $O
for i in 1 2 3; do
  for v in k4 k5; do
    if [ $v = k5 ]; then cd $R/ab_head; else cd $R; fi
    PYTHONPATH=$PWD timeout -k 10 120 python tools/kernel_bench.py --iters 30 > $O/${v}_$i.json 2> $O/${v}_$i.err
  done
done

# GPU tests of the touched paths, then a same-box A/B (ab_head = previous commit) of the
# host-cost probe and the 1080p headline, interleaved.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/ab3
mkdir -p $O
cd $R
PYTHONPATH=$R timeout -k 10 400 python -u -m pytest tests/test_transmux.py tests/test_e2e_gpu.py tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1
for i in 1 2 3; do
  for v in base new; do
    if [ $v = base ]; then cd $R/ab_head; else cd $R; fi
    PYTHONPATH=$PWD timeout -k 10 200 python bench.py --config hostcost --steps 60 --warmup 10 --verbose > $O/h_${v}_$i.log 2>&1
  done
done
cd $R
PYTHONPATH=$R timeout -k 10 200 python bench.py --verbose > $O/b1080_new.log 2>&1

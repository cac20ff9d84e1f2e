# Round-5 GPU pass: GPU tests, smoke, the N=1 headline once, and the N=8 exchange-overlap
# rehearsal (tools/overlap_n8.py, one run per mitigation).
#   bash tools/gpu_r5.sh            -> gpurun_out/r5/*.log
set -eo pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/${VAL_OUT:-r5}
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 300 python bench.py --verbose > $O/headline.log 2>&1
timeout -k 10 400 python -u tools/overlap_n8.py --iters 5 > $O/overlap_n8.log 2>&1
grep -h '^{' $O/headline.log | cut -c1-400
tail -1 $O/overlap_n8.log | cut -c1-300

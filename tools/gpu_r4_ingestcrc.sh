# A one-rank swarm skips the ingest CRC (no peer ever checks its trailers): GPU tests, then the
# HBM-origin probe (device-bound) and the headline with the pass skipped (default) and forced
# (HLSP2P_INGEST_CRC=1), interleaved:  bash tools/gpu_r4_ingestcrc.sh -> gpurun_out/r4_ingestcrc/*
set -eo pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/r4_ingestcrc
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1
for i in 1 2; do
  for f in 0 1; do
    HLSP2P_INGEST_CRC=$f timeout -k 10 300 python bench.py --ingest hbm --steps 100 --warmup 6 > $O/hbm_f${f}_$i.log 2>&1
  done
done
for f in 0 1; do
  HLSP2P_INGEST_CRC=$f timeout -k 10 300 python bench.py > $O/headline_f$f.log 2>&1
done
for f in $O/*.log; do case $f in *gpu_tests*) continue;; esac; echo "$f $(grep -h '^{' $f | python3 -c 'import json,sys; j=json.loads(sys.stdin.readline()); print(j["value"], j["ms_per_step"], j["per_rank"][0]["bound"])')"; done
tail -1 $O/gpu_tests.log

# Player-side cProfile (pure-Python players) of the HBM-origin fleet probe, short vs long run:
# what grows per fragment as the synthetic DVR playlist grows with the step count.
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/pprof
mkdir -p $O
HLSP2P_PLAYER_PROFILE=$O/s100 timeout -k 10 300 python bench.py --ingest hbm --steps 100 --warmup 5 --verbose > $O/s100.log 2>&1
HLSP2P_PLAYER_PROFILE=$O/s3000 timeout -k 10 400 python bench.py --ingest hbm --steps 3000 --warmup 5 --verbose > $O/s3000.log 2>&1

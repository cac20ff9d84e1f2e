# Config 5 at HBM scale: 4K 25 Mb/s AES segments through a 240 GB HBM arena (the ring wraps:
# ~26k x 12.5 MB segments = ~330 GB delivered), pinned-host CDN fallback.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/sat
timeout -k 10 300 python -u bench.py --config 4k25m --cache-gb 240 --steps 400 --warmup 10 --verbose > gpurun_out/sat/4k_240g.log 2>&1

# Per-GPU ceiling without the PCIe bound: the origin's segment pools live in HBM
# (bench.py --ingest hbm), so ingest is a device-to-device copy, as for segments that arrive
# over xGMI at N=8.  Plus the new fleet GPU test and a kernel-trace profile of the diagnostic.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/ingest_hbm
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_fleet.py -m gpu -x -v --timeout 240 --timeout-method thread > $O/fleet_gpu_test.log 2>&1
timeout -k 10 300 python bench.py --ingest hbm --steps 30 --warmup 5 --verbose > $O/hbm_p4.log 2>&1
timeout -k 10 300 python bench.py --ingest hbm --players 0 --steps 30 --warmup 5 --verbose > $O/hbm_p0.log 2>&1
timeout -k 10 300 python bench.py --ingest hbm --config 1080p6m-clear --steps 30 --warmup 5 --verbose > $O/hbm_clear_p4.log 2>&1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/pcie_p4.log 2>&1
timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $O/prof -o hbm -- python3 bench.py --ingest hbm --steps 20 --warmup 5 > $O/hbm_prof.log 2>&1

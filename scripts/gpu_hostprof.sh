# usage: bash scripts/gpu_hostprof.sh <tag>: stop_rate=1 PGD host/device split + cProfile, then a kernel trace of
# the C4 ADMM record (per-outer kernel list)
set -o pipefail
O=gpurun_out/${1:-hp}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python -u scripts/host_time_pgd_sr1.py > $O/sr1.log 2>&1 || exit $?
timeout -k 10 200 python -u scripts/host_prof_pgd_sr1.py >> $O/sr1.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/c4 -o run --output-format csv -- python3 bench.py --only c4 > $O/c4.log 2>&1 || exit $?
tail -60 $O/sr1.log

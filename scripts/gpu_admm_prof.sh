# C4 ADMM: bench line (GEMV pair vs one-pass normal operator) + rocprofv3 kernel trace/stats
set -o pipefail
O=gpurun_out/${1:-admm}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/bench_admm.py > $O/bench_admm.log 2>&1; echo "bench rc=$?"; tail -1 $O/bench_admm.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 scripts/bench_admm.py > $O/trace.log 2>&1; echo "trace rc=$?"
f=$(find $O/trace -name "*kernel_stats.csv" | head -1); head -20 "$f"

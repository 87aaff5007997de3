# PDS fused step: parity tests (fused PD3O / CV vs oracle and generic), C3 bench + kernel stats
set -o pipefail
O=gpurun_out/${1:-pdsq}
mkdir -p $O
export TMPDIR=/tmp
PT="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu"
timeout -k 10 600 $PT tests/test_gpu_pds_fused.py tests/test_gpu_bench_shapes.py tests/test_gpu_parity.py -k "pds or c3 or pd3o or condat or cv or PDS" > $O/tests.log 2>&1; echo "tests rc=$?"; tail -3 $O/tests.log
[ "${2:-}" = "tests" ] && exit 0
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 scripts/bench_pds.py > $O/bench.log 2>&1; echo "bench rc=$?"; grep '"algo"' $O/bench.log
f=$(find $O/trace -name "*kernel_stats.csv" | head -1); grep "pds_" "$f" | cut -c1-160

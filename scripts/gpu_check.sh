# usage: bash scripts/gpu_check.sh  -- gpu parity tests, smoke, bench (N=1), rocprof kernel-trace of the bench
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 \
 && echo "pytest ok" \
 && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 \
 && echo "smoke ok" \
 && timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1 \
 && tail -1 gpurun_out/bench.log \
 && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bench -o run --output-format csv -- python3 bench.py --cpu-seconds 0 > gpurun_out/prof_bench.log 2>&1 \
 && echo "prof ok"
rc=$?
tail -5 gpurun_out/pytest_gpu.log
exit $rc

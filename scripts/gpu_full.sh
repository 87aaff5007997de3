# usage: bash scripts/gpu_full.sh <tag> -- GPU parity suite, smoke, default bench line, then the rocprof
# kernel-trace/stats + PMC traffic passes (scripts/gpu_profile.sh).  Stops at the first failing step.
set -o pipefail
T=${1:-r01}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_$T.log 2>&1 \
 && tail -2 gpurun_out/pytest_gpu_$T.log \
 && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$T.log 2>&1 \
 && tail -1 gpurun_out/smoke_$T.log \
 && timeout -k 10 300 python bench.py > gpurun_out/bench_$T.jsonl 2> gpurun_out/bench_$T.err \
 && cat gpurun_out/bench_$T.jsonl \
 && bash scripts/gpu_profile.sh $T

set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1 \
  && tail -3 gpurun_out/pytest_gpu.log \
  && timeout -k 10 300 python bench.py --steps 300 --warmup 30 --cpu-iters 0 > gpurun_out/bench.log 2>&1 \
  && tail -2 gpurun_out/bench.log
rc=$?
tail -5 gpurun_out/pytest_gpu.log
exit $rc

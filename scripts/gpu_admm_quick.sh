set -o pipefail
mkdir -p gpurun_out/adm
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_gpu_dense_normal.py tests/test_gpu_bench_shapes.py -k "normal or admm or c4" -m gpu > gpurun_out/adm/tests.log 2>&1; echo "tests rc=$?"; tail -25 gpurun_out/adm/tests.log
timeout -k 10 300 python -u scripts/bench_admm.py > gpurun_out/adm/bench_admm.log 2>&1; echo "bench rc=$?"; tail -3 gpurun_out/adm/bench_admm.log

# CG p-fold: parity tests and the c4 leg with the fold on / off (PXA_CG_FOLD_P), interleaved
set -o pipefail
O=gpurun_out/${1:-r06an}; mkdir -p $O
PT="python -u -m pytest -v --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 900 $PT -m gpu tests/test_gpu_dense_normal.py tests/test_gpu_admm_fused.py tests/test_gpu_bench_shapes.py tests/test_gpu_distributed.py tests/test_gpu_rccl.py -k "normal or cg or admm or c4 or rccl or dense" > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log; [ $rc -le 1 ] || exit $rc
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --only c4 > $O/fold_$i.log 2>&1 || exit $?
  PXA_CG_FOLD_P=0 timeout -k 10 300 python3 bench.py --only c4 > $O/nofold_$i.log 2>&1 || exit $?
done

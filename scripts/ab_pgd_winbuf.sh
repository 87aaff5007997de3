# A/B: interior window loads as buffer loads (ab/libpyxu_amd_buf.so) against global loads (default), parity + timing
set -o pipefail
O=gpurun_out/${1:-r06aw}; mkdir -p $O
PXA_LIB_PATH=ab/libpyxu_amd_buf.so timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests/test_gpu_pgd_variants.py -k "vector_and_scalar or pipe_kernel_matches" > $O/tests.log 2>&1; rc=$?; tail -1 $O/tests.log; [ $rc -le 1 ] || exit $rc
DRV="python3 bench.py --steps 20 --warmup 5 --no-sub --cpu-seconds 0"
for i in 1 2 3; do
  timeout -k 10 120 $DRV > $O/def_$i.log 2>&1 || exit $?
  PXA_LIB_PATH=ab/libpyxu_amd_buf.so timeout -k 10 120 $DRV > $O/buf_$i.log 2>&1 || exit $?
done
timeout -k 10 300 python3 bench.py --only c2_4096 > $O/def_4096.log 2>&1 || exit $?
PXA_LIB_PATH=ab/libpyxu_amd_buf.so timeout -k 10 300 python3 bench.py --only c2_4096 > $O/buf_4096.log 2>&1 || exit $?

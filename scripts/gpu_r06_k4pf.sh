# K4 one-row kernel with next-plane prefetch (PXA_TUNE_DUAL_ROWS = 3) against the default, interleaved
set -o pipefail
O=gpurun_out/${1:-r06ar}; mkdir -p $O
PT="python -u -m pytest -v --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 600 $PT -m gpu tests/test_gpu_pds_fused.py -k "tv_dual" > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log; [ $rc -le 1 ] || exit $rc
for i in 1 2 3; do
  timeout -k 10 300 python3 bench.py --only k4 > $O/base_$i.log 2>&1 || exit $?
  PXA_TUNE=11=3 timeout -k 10 300 python3 bench.py --only k4 > $O/pf_$i.log 2>&1 || exit $?
done

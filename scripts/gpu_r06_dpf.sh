# kernel D plane prefetch (PXA_TUNE_PDS_MARCH bit 8): parity, then the c3 leg on / off, interleaved
set -o pipefail
O=gpurun_out/${1:-r06ao}; mkdir -p $O
PT="python -u -m pytest -v --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 900 $PT -m gpu tests/test_gpu_pds_fused.py -k "prefetch or lookahead_matches" > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log; [ $rc -le 1 ] || exit $rc
for i in 1 2; do
  timeout -k 10 400 python3 bench.py --only c3 --c3-cpu-n 0 > $O/base_$i.log 2>&1 || exit $?
  PXA_TUNE=7=256 timeout -k 10 400 python3 bench.py --only c3 --c3-cpu-n 0 > $O/nopf_$i.log 2>&1 || exit $?
  PXA_TUNE=7=512 timeout -k 10 400 python3 bench.py --only c3 --c3-cpu-n 0 > $O/pf2_$i.log 2>&1 || exit $?
done

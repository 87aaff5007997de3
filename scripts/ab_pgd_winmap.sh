# A/B: tile-first window order (default) against the row-major order of rounds 1-5 (ab/libpyxu_amd_rm.so), interleaved
set -o pipefail
O=gpurun_out/${1:-r06am}; mkdir -p $O
DRV="python3 bench.py --steps 20 --warmup 5 --no-sub --cpu-seconds 0"
for i in 1 2 3; do
  timeout -k 10 120 $DRV > $O/new_$i.log 2>&1 || exit $?
  PXA_LIB_PATH=ab/libpyxu_amd_rm.so timeout -k 10 120 $DRV > $O/rm_$i.log 2>&1 || exit $?
done
timeout -k 10 300 python3 bench.py --only c2_4096 > $O/new_4096.log 2>&1 || exit $?
PXA_LIB_PATH=ab/libpyxu_amd_rm.so timeout -k 10 300 python3 bench.py --only c2_4096 > $O/rm_4096.log 2>&1 || exit $?

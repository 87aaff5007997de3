# kernel D: one plane ahead (default) against two (PXA_TUNE_PDS_MARCH bit 9), interleaved, 3 rounds
set -o pipefail
O=gpurun_out/${1:-r06aq}; mkdir -p $O
for i in 1 2 3; do
  timeout -k 10 400 python3 bench.py --only c3 --c3-cpu-n 0 > $O/base_$i.log 2>&1 || exit $?
  PXA_TUNE=7=512 timeout -k 10 400 python3 bench.py --only c3 --c3-cpu-n 0 > $O/pf2_$i.log 2>&1 || exit $?
done

# A/B of the PGD tile kernel's TV-exchange build (csrc/Makefile ab AB_TAG=tvx AB_FLAGS=-DPXA_PGD_TVX=1) against
# the same tree built plainly (AB_TAG=base): bits first (10 steps at 2048^2 and at 1000 x 1500, edge tiles),
# then the parity tests under the variant, then interleaved timings.
export TMPDIR=/tmp; O=gpurun_out/${TAG:-tvx}; mkdir -p $O
for v in base tvx; do
  PXA_LIB_PATH=ab/libpyxu_amd_$v.so timeout -k 10 200 python3 scripts/pgd_bits_dump.py $O/bits_$v.npz > $O/bits_$v.log 2>&1 || exit 1
done
python3 -c "
import numpy as np
a, b = np.load('$O/bits_base.npz'), np.load('$O/bits_tvx.npz')
for k in a.files:
    print(k, 'bit-identical' if np.array_equal(a[k].view(np.uint32), b[k].view(np.uint32)) else 'DIFFER max %g' % np.max(np.abs(a[k] - b[k])))
"
PXA_LIB_PATH=ab/libpyxu_amd_tvx.so timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu tests/test_gpu_pgd_variants.py tests/test_gpu_parity.py tests/test_gpu_bench_shapes.py -k "pgd or PGD or c2 or c5" > $O/tests.log 2>&1; tail -1 $O/tests.log
DRV="python3 bench.py --steps 20 --warmup 5 --no-sub --cpu-seconds 0"
for i in 1 2 3; do
  for v in base tvx; do
    PXA_LIB_PATH=ab/libpyxu_amd_$v.so timeout -k 10 120 $DRV > $O/drv_${v}_$i.log 2>&1 || exit 1
    echo "drv $v $i $(grep -h '^{' $O/drv_${v}_$i.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["roofline"]["kernel_ms"])')"
  done
done
for v in base tvx; do
  PXA_LIB_PATH=ab/libpyxu_amd_$v.so timeout -k 10 300 python3 bench.py --only c5 > $O/c5_$v.log 2>&1 || exit 1
  echo "c5 $v $(grep -h '^{' $O/c5_$v.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["roofline"]["kernel_ms"])')"
  PXA_LIB_PATH=ab/libpyxu_amd_$v.so timeout -k 10 300 python3 bench.py --only c2_4096 > $O/c4096_$v.log 2>&1 || exit 1
  echo "4096 $v $(grep -h '^{' $O/c4096_$v.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["roofline"]["kernel_ms"])')"
done

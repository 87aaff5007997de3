export TMPDIR=/tmp; O=gpurun_out/${TAG:-r06b}; mkdir -p $O
DRV="python3 bench.py --steps 20 --warmup 5 --no-sub --cpu-seconds 0"
for i in 1 2; do
  for v in base ilp mem bias; do
    PXA_LIB_PATH=ab/libpyxu_amd_$v.so timeout -k 10 120 $DRV > $O/drv_${v}_$i.log 2>&1 || exit 1
    echo "drv $v $i $(grep -h '^{' $O/drv_${v}_$i.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["roofline"]["kernel_ms"])')"
  done
done
for v in base ilp mem bias; do
  PXA_LIB_PATH=ab/libpyxu_amd_$v.so timeout -k 10 300 python3 bench.py --only c5 > $O/c5_$v.log 2>&1 || exit 1
  echo "c5 $v $(grep -h '^{' $O/c5_$v.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["roofline"]["kernel_ms"])')"
  PXA_LIB_PATH=ab/libpyxu_amd_$v.so timeout -k 10 300 python3 bench.py --only c2_4096 > $O/c4096_$v.log 2>&1 || exit 1
  echo "4096 $v $(grep -h '^{' $O/c4096_$v.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["roofline"]["kernel_ms"])')"
done

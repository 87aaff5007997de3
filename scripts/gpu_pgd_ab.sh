# usage: bash scripts/gpu_pgd_ab.sh <tag> -- PGD kernel variants: bit-exactness tests, PGD parity tests,
# A/B bench lines (persistent LDS-DMA vs tile kernel), rocprofv3 kernel trace of both.
set -o pipefail
T=${1:-ab}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
step() {
  local name=$1 lim=$2; shift 2
  echo "== $name"
  timeout -k 10 $lim "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "   rc=$rc"; tail -4 $O/$name.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
PT="python -u -m pytest -v --timeout 300 --timeout-method thread -p no:cacheprovider"
step variants 300 $PT tests/test_gpu_pgd_variants.py -m gpu
step pgdtests 600 $PT tests/test_gpu_bench_shapes.py tests/test_gpu_parity.py -m gpu -k "pgd or c1 or c2 or c5 or batch or fused"
for k in 0 5; do step bench_k$k 200 python bench.py --no-sub --cpu-seconds 0 --pgd-kernel $k; done
step trace 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 bench.py --no-sub --cpu-seconds 0 --steps 200 --warmup 20
grep pgd_tv2d $O/trace/run_kernel_stats.csv | cut -c1-250
echo done

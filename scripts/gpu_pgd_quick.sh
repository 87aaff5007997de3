# usage: bash scripts/gpu_pgd_quick.sh <tag> [kernel values...] -- variant bit-exactness + A/B bench
# lines of the PGD kernel variants (PXA_TUNE_PGD_KERNEL values, default "0 5")
set -o pipefail
T=${1:-q}
shift
KS=${@:-0 5}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_pgd_variants.py -m gpu > $O/variants.log 2>&1; rc=$?; tail -2 $O/variants.log
[ $rc -le 1 ] || exit $rc
for k in $KS; do timeout -k 10 200 python bench.py --no-sub --cpu-seconds 0 --pgd-kernel $k > $O/bench_k$k.log 2>&1 || exit $?; grep -o '"kernel_ms": [0-9.]*' $O/bench_k$k.log | sed "s/^/k$k /"; done

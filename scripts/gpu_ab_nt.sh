# A/B: PGD tile kernel default vs streaming epilogue (--pgd-kernel 6); dense GEMV with streaming A loads
set -o pipefail
O=gpurun_out/nt
mkdir -p $O
export TMPDIR=/tmp
PT="python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu"
timeout -k 10 300 $PT tests/test_gpu_dense_normal.py tests/test_gpu_parity.py -k "dense or admm or normal" > $O/tests.log 2>&1; echo "tests rc=$?"; tail -2 $O/tests.log
for k in 0 6 0 6; do
  timeout -k 10 120 python bench.py --no-sub --cpu-seconds 0 --pgd-kernel $k > $O/b$k.log 2>&1 || exit 1
  python -c "import json,sys; d=json.loads(open('$O/b$k.log').read().strip().splitlines()[-1]); print('kernel $k', d['value'], d['roofline']['kernel_ms'])"
done
timeout -k 10 300 python -u scripts/bench_admm.py > $O/admm.log 2>&1; echo "admm rc=$?"; tail -1 $O/admm.log

# PGD / PDS tile-kernel change check: parity subset, headline bench (no sub-records), SQ LDS counters
set -o pipefail
O=gpurun_out/${1:-pgdc}
mkdir -p $O
export TMPDIR=/tmp
PT="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu"
timeout -k 10 600 $PT tests/test_gpu_parity.py tests/test_gpu_pds_fused.py tests/test_gpu_bench_shapes.py tests/test_gpu_pgd_variants.py > $O/tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do timeout -k 10 120 python bench.py --no-sub --cpu-seconds 0 > $O/bench$i.log 2>&1 || exit 1; python -c "import json; d=json.loads(open('$O/bench$i.log').read().strip().splitlines()[-1]); print('bench', d['value'], d['roofline']['kernel_ms'])"; done
timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY --kernel-trace -d $O/sq1 -o run --output-format csv -- python3 bench.py --no-sub --cpu-seconds 0 --steps 20 --warmup 5 --prime-seconds 0 > $O/sq1.log 2>&1 || exit 1
python3 scripts/pmc_summary.py $O/sq1 pgd_tv2d
[ "${2:-}" = "pds" ] && PXA_N=1024 PXA_GENERIC_N=0 timeout -k 10 300 python scripts/bench_pds.py > $O/pds.log 2>&1 && grep algo $O/pds.log
exit 0

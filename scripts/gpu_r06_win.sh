# tile-first window mapping: PGD parity + lag tests, headline A/B against the r06x figures, stop_rate-1 timing
set -o pipefail
O=gpurun_out/${1:-r06ac}; mkdir -p $O
PT="python -u -m pytest -v --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 900 $PT -m gpu tests/test_gpu_pgd_variants.py tests/test_gpu_parity.py tests/test_gpu_bench_shapes.py tests/test_gpu_solver_lag.py tests/test_gpu_solver_engine.py -k "pgd or c2 or c5 or trajectory or strip or pipe or lag or speculative or fold or relerr or smoke" > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log; [ $rc -le 1 ] || exit $rc
for i in 1 2 3; do timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 --no-sub --cpu-seconds 0 > $O/drv_$i.log 2>&1 || exit $?; done
timeout -k 10 200 python3 scripts/host_time_pgd_sr1.py 2048 > $O/ht2048.log 2>&1

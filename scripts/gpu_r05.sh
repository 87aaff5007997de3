# usage: bash scripts/gpu_r05.sh <tag> <stage>
# GPU calls of round 5.  Stages:
#   new    the tests added / touched this round, the default bench line, a kernel trace of the headline
#   full   the whole -m gpu suite, smoke, the default bench line
#   prof   rocprofv3 kernel trace (--stats) of the headline + the PGD PMC passes (traffic, occupancy, waits)
#   c3prof kernel-D / B PMC traffic passes at 1024^3 + the c3 record
# Test failures (rc 1) do not stop the run; any other failure (fault, abort, timeout) ends it there.
set -o pipefail
T=${1:-r05}
S=${2:-new}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
step() {  # step <name> <timeout> <cmd...>: run with a time limit; stop the script unless rc in {0, 1}
  local name=$1 lim=$2; shift 2
  echo "== $name"
  timeout -k 10 $lim "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "   rc=$rc"; tail -3 $O/$name.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
PT="python -u -m pytest -v --timeout 300 --timeout-method thread -p no:cacheprovider"
P=$O/prof
mkdir -p $P
DRV="python3 bench.py --steps 20 --warmup 5 --no-sub --cpu-seconds 0"
export PXA_FAIL_DIR=$O/fail
pmc_pgd() {  # the headline's PGD counters, one pass each (separate runs: FETCH / WRITE / SQ)
  step pgdfetch 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $P/pgdfetch -o run --output-format csv -- $DRV
  step pgdwrite 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $P/pgdwrite -o run --output-format csv -- $DRV
  step pgdsq 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS --kernel-trace -d $P/pgdsq -o run --output-format csv -- $DRV
  step pgdsq2 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_ACTIVE_INST_ANY SQ_BUSY_CU_CYCLES --kernel-trace -d $P/pgdsq2 -o run --output-format csv -- $DRV
  python3 scripts/pmc_traffic.py $P/pgdfetch $P/pgdwrite "pgd_tv2d_kernel" pgd_tv2d_kernel@2048x2048 $P/traffic_pgd.json $T || true
}
if [ "$S" = "new" ]; then
  step newtests 900 $PT -m gpu tests/test_gpu_c3_fullsize.py tests/test_gpu_fft.py tests/test_gpu_stencil_fft.py \
       tests/test_gpu_dense_normal.py tests/test_gpu_solver_engine.py
  step drv1 120 $DRV
  step trace 120 rocprofv3 --kernel-trace --stats -d $P/trace -o run --output-format csv -- $DRV
  step bench 900 python bench.py --steps 20 --warmup 5
fi
if [ "$S" = "admm" ]; then
  step admmtests 600 $PT -m gpu tests/test_gpu_admm_fused.py tests/test_gpu_dense_normal.py
  step admmtests2 900 $PT -m gpu tests/test_gpu_pds_fused.py tests/test_gpu_parity.py tests/test_gpu_solver_engine.py tests/test_gpu_blocks.py tests/test_gpu_long_trajectories.py
  step c4a 300 python3 bench.py --only c4
  step c4b 300 python3 bench.py --only c4
  step c4trace 300 rocprofv3 --kernel-trace --stats -d $P/c4 -o run --output-format csv -- python3 bench.py --only c4
  python3 scripts/c4_timeline.py $P/c4 > $O/c4timeline.log 2>&1 || true
fi
if [ "$S" = "couple" ]; then
  step ctests 600 $PT -m gpu tests/test_gpu_pds_fused.py -k "coupled or persistent or lookahead_matches"
  step c3base 300 python3 bench.py --only c3
  PXA_TUNE=7=4 step c3c0 300 python3 bench.py --only c3
  PXA_TUNE=7=68 step c3c8 300 python3 bench.py --only c3
  PXA_TUNE=7=20 step c3c2 300 python3 bench.py --only c3
  step c3base2 300 python3 bench.py --only c3
  B3="python3 bench.py --only c3 --c3-steps 3"
  PXA_TUNE=7=4 step fetchc3c 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $P/fetchc3c -o run --output-format csv -- $B3
  PXA_TUNE=7=4 step writec3c 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $P/writec3c -o run --output-format csv -- $B3
  python3 scripts/pmc_traffic.py $P/fetchc3c $P/writec3c "pds_march_kernel<float, 6, 1, true, false, true, true, true>" pds_march_kernel_pd3o_coupled@1024^3 $P/traffic_c3c.json $T || true
fi
if [ "$S" = "a" ]; then
  step pgdtests 600 $PT -m gpu tests/test_gpu_pgd_variants.py tests/test_gpu_bench_shapes.py tests/test_gpu_long_trajectories.py tests/test_gpu_small_weights.py -k "pgd or c2 or c5"
  step drvnew 120 $DRV
  PXA_TUNE=0=1 step drvold 120 $DRV
  step drvnew2 120 $DRV
  PXA_TUNE=0=1 step drvold2 120 $DRV
  step c5new 300 python3 bench.py --only c5
  PXA_TUNE=0=1 step c5old 300 python3 bench.py --only c5
  step c4096new 300 python3 bench.py --only c2_4096
  PXA_TUNE=0=1 step c4096old 300 python3 bench.py --only c2_4096
  step trace 120 rocprofv3 --kernel-trace --stats -d $P/trace -o run --output-format csv -- $DRV
  step newtests 900 $PT -m gpu tests/test_gpu_c3_fullsize.py tests/test_gpu_fft.py tests/test_gpu_stencil_fft.py \
       tests/test_gpu_dense_normal.py tests/test_gpu_solver_engine.py
fi
if [ "$S" = "b" ]; then
  step newtests 900 $PT -m gpu tests/test_gpu_c3_fullsize.py tests/test_gpu_fft.py tests/test_gpu_stencil_fft.py \
       tests/test_gpu_dense_normal.py tests/test_gpu_solver_engine.py tests/test_gpu_pgd_variants.py
  step drv1 120 $DRV
  step drv2 120 $DRV
  step trace 120 rocprofv3 --kernel-trace --stats -d $P/trace -o run --output-format csv -- $DRV
  step bench 900 python bench.py --steps 20 --warmup 5
fi
if [ "$S" = "c" ]; then
  step tests 900 $PT -m gpu tests/test_gpu_fft.py tests/test_gpu_c3_fullsize.py tests/test_gpu_pds_fused.py tests/test_gpu_long_trajectories.py tests/test_gpu_bench_shapes.py
  step c3new 300 python3 bench.py --only c3
  PXA_TUNE=7=2 step c3old 300 python3 bench.py --only c3
  step c3new2 300 python3 bench.py --only c3
  B3="python3 bench.py --only c3 --c3-steps 3"
  step fetchc3 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $P/fetchc3 -o run --output-format csv -- $B3
  step writec3 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $P/writec3 -o run --output-format csv -- $B3
  python3 scripts/pmc_traffic.py $P/fetchc3 $P/writec3 "pds_march_kernel<float, 6, 1, true, false, true, true>" pds_march_kernel_pd3o@1024^3 $P/traffic_c3.json $T || true
  python3 scripts/pmc_traffic.py $P/fetchc3 $P/writec3 "pds_march_kernel<float, 6, 1, false, false, true, true>" pds_march_kernel_cv@1024^3 $P/traffic_c3.json $T || true
fi
if [ "$S" = "d" ]; then
  step pdstests 600 $PT -m gpu tests/test_gpu_pds_fused.py -k "persistent or two_positions or lookahead_matches"
  step sr1time 300 python3 scripts/host_time_pgd_sr1.py
  step sr1prof 300 python3 scripts/prof_sr1.py
  step trace 120 rocprofv3 --kernel-trace --stats -d $P/trace -o run --output-format csv -- $DRV
  pmc_pgd
fi
if [ "$S" = "e" ]; then
  step tests 900 $PT -m gpu tests/test_gpu_pgd_variants.py tests/test_gpu_solver_engine.py tests/test_gpu_parity.py tests/test_gpu_bench_shapes.py tests/test_gpu_long_trajectories.py tests/test_gpu_small_weights.py tests/test_gpu_distributed.py
  step sr1time 300 python3 scripts/host_time_pgd_sr1.py
  step sr1prof 300 python3 scripts/prof_sr1.py
  step drv1 120 $DRV
  step drv2 120 $DRV
  step bench 900 python bench.py --steps 20 --warmup 5
fi
if [ "$S" = "f" ]; then
  step foldtest 300 $PT -m gpu tests/test_gpu_pgd_variants.py
  PXA_RELERR_SINK=1 step foldtest_sink 300 $PT -m gpu tests/test_gpu_pgd_variants.py tests/test_gpu_solver_engine.py
  step foldlat 120 python3 scripts/fold_latency.py
  step sr1time 300 python3 scripts/host_time_pgd_sr1.py
  PXA_RELERR_SINK=1 step sr1time_sink 300 python3 scripts/host_time_pgd_sr1.py
  step drv1 120 $DRV
fi
if [ "$S" = "g" ] || [ "$S" = "h" ]; then
  step pgdtests 600 $PT -m gpu tests/test_gpu_pgd_variants.py tests/test_gpu_bench_shapes.py tests/test_gpu_parity.py tests/test_gpu_long_trajectories.py tests/test_gpu_small_weights.py -k "pgd or c2 or c5 or smoke or trajectory"
  for i in 1 2; do
    for v in base unit ctv; do PXA_LIB_PATH=ab/libpyxu_amd_$v.so step drv_${v}_$i 120 $DRV; done
    step drv_main_$i 120 $DRV
  done
  for v in base unit ctv; do PXA_LIB_PATH=ab/libpyxu_amd_$v.so step c5_$v 300 python3 bench.py --only c5; done
  step c5_main 300 python3 bench.py --only c5
  step trace 120 rocprofv3 --kernel-trace --stats -d $P/trace -o run --output-format csv -- $DRV
fi
if [ "$S" = "g" ] || [ "$S" = "h" ]; then
  if [ "$S" = "h" ]; then
    step c4 300 python3 bench.py --only c4
    step c4hostprof 300 python3 scripts/c4_host_prof.py
    step c4trace 300 rocprofv3 --kernel-trace --stats -d $P/c4 -o run --output-format csv -- python3 bench.py --only c4
    python3 scripts/c4_timeline.py $P/c4 > $O/c4timeline.log 2>&1 || true
  fi
fi
if [ "$S" = "pgd" ]; then
  step pgdtests 600 $PT -m gpu tests/test_gpu_pgd_variants.py tests/test_gpu_bench_shapes.py tests/test_gpu_parity.py -k "pgd or c2 or c5 or smoke or trajectory"
  step drv1 120 $DRV
  step drv2 120 $DRV
  step c5 300 python3 bench.py --only c5
  step trace 120 rocprofv3 --kernel-trace --stats -d $P/trace -o run --output-format csv -- $DRV
fi
if [ "$S" = "prof" ]; then
  step trace 120 rocprofv3 --kernel-trace --stats -d $P/trace -o run --output-format csv -- $DRV
  pmc_pgd
fi
if [ "$S" = "c3prof" ]; then
  step c3 300 python3 bench.py --only c3
  B3="python3 bench.py --only c3 --c3-steps 3"
  step fetchc3 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $P/fetchc3 -o run --output-format csv -- $B3
  step writec3 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $P/writec3 -o run --output-format csv -- $B3
  python3 scripts/pmc_traffic.py $P/fetchc3 $P/writec3 "pds_march_kernel<float, 6, 1, true, false, true, true>" pds_march_kernel_pd3o@1024^3 $P/traffic_c3.json $T || true
  python3 scripts/pmc_traffic.py $P/fetchc3 $P/writec3 "pds_march_kernel<float, 6, 1, false, false, true, true>" pds_march_kernel_cv@1024^3 $P/traffic_c3.json $T || true
fi
if [ "$S" = "full" ]; then
  step pytest 1200 $PT tests -m gpu
  step smoke 150 python -c "import __graft_entry__ as g; g.smoke()"
fi
if [ "$S" = "bench" ]; then
  step bench 1000 python bench.py --steps 20 --warmup 5
fi
echo done

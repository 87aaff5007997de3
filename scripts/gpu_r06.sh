# usage: bash scripts/gpu_r06.sh <tag> <stage>
# GPU calls of round 6.  Stages:
#   new    the tests added / touched this round, the default driver bench line, a kernel trace of the headline
#   full   the whole -m gpu suite + smoke
#   bench  the default bench line (all sub-records)
#   prof   rocprofv3 kernel trace (--stats) of the headline + the PGD PMC passes (traffic, occupancy, waits)
#   c3prof / k4prof  kernel traces + traffic PMC passes of the C3 / K4 legs
# Test failures (rc 1) do not stop the run; any other failure (fault, abort, timeout) ends it there.
set -o pipefail
T=${1:-r06}
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
  python3 scripts/pmc_traffic.py $P/pgdfetch $P/pgdwrite "pgd_tv2d_kernel<float, 6>" pgd_tv2d_kernel@2048x2048 $P/traffic_pgd.json $T || true
  python3 scripts/pmc_sum.py "pgd_tv2d_kernel<float, 6>" $P/pgdfetch $P/pgdwrite $P/pgdsq $P/pgdsq2 > $O/pmc_summary.txt 2>&1 || true
}
if [ "$S" = "new" ]; then
  step newtests 900 $PT -m gpu tests/test_gpu_rccl.py tests/test_gpu_fft.py tests/test_gpu_solver_engine.py \
       tests/test_gpu_admm_fused.py tests/test_gpu_dense_normal.py tests/test_gpu_distributed.py
  step drv1 120 $DRV
  step trace 120 rocprofv3 --kernel-trace --stats -d $P/trace -o run --output-format csv -- $DRV
fi
if [ "$S" = "strip" ]; then
  step pgdtests 900 $PT -m gpu tests/test_gpu_pgd_variants.py tests/test_gpu_bench_shapes.py tests/test_gpu_parity.py -k "pgd or c2 or c5 or smoke or trajectory or strip"
  for i in 1 2; do
    step drv_strip_$i 120 $DRV
    PXA_TUNE=0=1 step drv_tile_$i 120 $DRV
  done
  step c5_strip 300 python3 bench.py --only c5
  PXA_TUNE=0=1 step c5_tile 300 python3 bench.py --only c5
  step c4096_strip 300 python3 bench.py --only c2_4096
  PXA_TUNE=0=1 step c4096_tile 300 python3 bench.py --only c2_4096
  step trace 120 rocprofv3 --kernel-trace --stats -d $P/trace -o run --output-format csv -- $DRV
fi
if [ "$S" = "pipe" ]; then  # the pipelined PGD kernel (PXA_TUNE 12=1) against the tile kernel (default)
  step pipetests 600 $PT -m gpu tests/test_gpu_pgd_variants.py
  for i in 1 2; do
    PXA_TUNE=12=1 step drv_pipe_$i 120 $DRV
    step drv_tile_$i 120 $DRV
  done
fi
if [ "$S" = "subtraffic" ]; then  # round-current traffic passes of the c2_4096 and c5 sub-records
  for leg in c2_4096:pgd_tv2d_kernel@4096x4096 c5:pgd_tv2d_kernel@512x512x512; do
    o=${leg%%:*}; key=${leg##*:}
    step fetch_$o 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $P/fetch_$o -o run --output-format csv -- python3 bench.py --only $o
    step write_$o 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $P/write_$o -o run --output-format csv -- python3 bench.py --only $o
    python3 scripts/pmc_traffic.py $P/fetch_$o $P/write_$o "pgd_tv2d_kernel<float, 6>" $key $P/traffic_sub.json $T || true
  done
fi
if [ "$S" = "c4mfma" ]; then  # round-current PMC passes of the c4 operator kernel and the dense MFMA kernels
  step fetch_c4 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $P/fetch_c4 -o run --output-format csv -- python3 bench.py --only c4
  step write_c4 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $P/write_c4 -o run --output-format csv -- python3 bench.py --only c4
  python3 scripts/pmc_traffic.py $P/fetch_c4 $P/write_c4 "normal_group_kernel" normal_group_kernel@8192x65536 $P/traffic_c4.json $T || true
  step mfma 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace -d $P/mfma -o run --output-format csv -- python3 bench.py --only dense_mfma
  python3 scripts/pmc_mfma.py $P/mfma $P/mfma_busy.json $T > $O/mfma.txt 2>&1 || true
fi
if [ "$S" = "k4" ]; then
  step k4tests 600 $PT -m gpu tests/test_gpu_pds_fused.py -k "tv_dual"
  for i in 1 2; do
    for v in 0 2 4; do PXA_TUNE=11=$v step k4_rows${v}_$i 300 python3 bench.py --only k4; done
  done
  K4="python3 bench.py --only k4 --k4-which 3d"
  for v in 0 2 4; do
    PXA_TUNE=11=$v step k4fetch$v 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $P/k4fetch$v -o run --output-format csv -- $K4
    PXA_TUNE=11=$v step k4write$v 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $P/k4write$v -o run --output-format csv -- $K4
  done
  python3 scripts/pmc_traffic.py $P/k4fetch0 $P/k4write0 "pds_dual_kernel" pds_dual_kernel@1024x1024x1024 $P/traffic_k4.json $T || true
  python3 scripts/pmc_traffic.py $P/k4fetch2 $P/k4write2 "pds_dual_rows_kernel<float, 4, 2," pds_dual_rows_kernel_rb2@1024x1024x1024 $P/traffic_k4.json $T || true
  python3 scripts/pmc_traffic.py $P/k4fetch4 $P/k4write4 "pds_dual_rows_kernel<float, 4, 4," pds_dual_rows_kernel_rb4@1024x1024x1024 $P/traffic_k4.json $T || true
fi
if [ "$S" = "c3prof" ]; then
  step c3 600 python3 bench.py --only c3
  step c3trace 600 rocprofv3 --kernel-trace --stats -d $P/c3trace -o run --output-format csv -- python3 bench.py --only c3
  step k4 300 python3 bench.py --only k4
  step k4trace 300 rocprofv3 --kernel-trace --stats -d $P/k4trace -o run --output-format csv -- python3 bench.py --only k4
  B3="python3 bench.py --only c3 --c3-steps 3"
  step fetchc3 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $P/fetchc3 -o run --output-format csv -- $B3
  step writec3 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $P/writec3 -o run --output-format csv -- $B3
  for k in "pds_plane_kernel<float, 6, 0>:pds_plane_kernel_pd3o@1024^3" "pds_plane_kernel<float, 6, 2>:pds_plane_kernel_cv@1024^3" \
           "pds_march_kernel<float, 6, 1, true, false, true, true, false, 1>:pds_march_kernel_pd3o@1024^3" \
           "pds_march_kernel<float, 6, 1, false, false, true, true, false, 1>:pds_march_kernel_cv@1024^3"; do
    python3 scripts/pmc_traffic.py $P/fetchc3 $P/writec3 "${k%%:*}" "${k##*:}" $P/traffic_c3.json $T || true
  done
  K42="python3 bench.py --only k4 --k4-which 2d"
  step fetchk4 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $P/fetchk4 -o run --output-format csv -- $K42
  step writek4 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $P/writek4 -o run --output-format csv -- $K42
  python3 scripts/pmc_traffic.py $P/fetchk4 $P/writek4 "pds_dual_kernel" pds_dual_kernel@2048x2048 $P/traffic_c3.json $T || true
fi
if [ "$S" = "lag" ]; then
  step lagtests 900 $PT -m gpu tests/test_gpu_solver_lag.py tests/test_gpu_solver_engine.py tests/test_gpu_pgd_variants.py -k "lag or speculative or fold or relerr or async or objective"
  step sr1ab 600 python3 scripts/sr1_lag_ab.py 400
fi
if [ "$S" = "sr1" ]; then
  step striptest 300 $PT -m gpu tests/test_gpu_pgd_variants.py -k "strip_kernel_solver"
  SR1_ARMS=short step sr1_20 300 python3 scripts/sr1_lag_ab.py 20
  SR1_ARMS=short step sr1_100 300 python3 scripts/sr1_lag_ab.py 100
fi
if [ "$S" = "full" ]; then
  step pytest 1200 $PT tests -m gpu
  step smoke 150 python -c "import __graft_entry__ as g; g.smoke()"
fi
if [ "$S" = "bench" ]; then
  step bench 1000 python bench.py --steps 20 --warmup 5
fi
if [ "$S" = "prof" ]; then
  step trace 120 rocprofv3 --kernel-trace --stats -d $P/trace -o run --output-format csv -- $DRV
  pmc_pgd
fi

if [ "$S" = "k4lds" ]; then  # plane-block kernel C (PXA_TUNE 11=8) against the one-row kernel
  step k4tests 600 $PT -m gpu tests/test_gpu_pds_fused.py -k "tv_dual"
  for i in 1 2; do
    step k4_one_$i 300 python3 bench.py --only k4 --k4-which 3d
    PXA_TUNE=11=8 step k4_lds_$i 300 python3 bench.py --only k4 --k4-which 3d
    PXA_TUNE=11=9 step k4_ldsz_$i 300 python3 bench.py --only k4 --k4-which 3d
  done
  K4="python3 bench.py --only k4 --k4-which 3d"
  PXA_TUNE=11=8 step k4fetch8 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $P/k4fetch8 -o run --output-format csv -- $K4
  PXA_TUNE=11=8 step k4write8 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $P/k4write8 -o run --output-format csv -- $K4
  python3 scripts/pmc_traffic.py $P/k4fetch8 $P/k4write8 "pds_dual_lds_kernel" pds_dual_lds_kernel@1024x1024x1024 $P/traffic_k4.json $T || true
fi
echo done

# usage: bash scripts/gpu_r04.sh <tag> <stage>
# GPU calls of round 4.  Stages:
#   new    the tests added this round, the k4 / dense_mfma records, the headline at the driver's flags,
#          the counter list, k4 traffic and dense MFMA-busy passes
#   full   the whole -m gpu suite, smoke, the default bench line
#   prof   rocprofv3 kernel trace of the headline + the PMC passes of profiles/ (traffic, SQ, MFMA busy)
# Test failures (rc 1) do not stop the run; any other failure (fault, abort, timeout) ends it there.
set -o pipefail
T=${1:-r04}
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
if [ "$S" = "new" ]; then
  export PXA_PARITY_RECORD=$O/small_weights.jsonl
  step newtests 900 $PT -m gpu tests/test_gpu_small_weights.py tests/test_gpu_directional.py tests/test_gpu_distributed.py \
       tests/test_gpu_solver_engine.py "tests/test_gpu_pds_fused.py::test_tv_dual_update_vs_oracle" \
       "tests/test_gpu_parity.py::test_dense_mfma_vs_fp64" "tests/test_gpu_parity.py::test_dense_lds_kernel_matches_register_kernel"
  unset PXA_PARITY_RECORD
  step k4 300 python3 bench.py --only k4
  step dense 300 python3 bench.py --only dense_mfma
  step densereg 300 python3 scripts/bench_dense.py
  step drv1 120 $DRV
  step drv2 120 $DRV
  step drv3 120 $DRV
  step long 120 python3 bench.py --steps 200 --warmup 20 --no-sub --cpu-seconds 0
  step list 120 rocprofv3 -L
  for w in 2d 3d; do
    step k4fetch$w 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $P/k4fetch$w -o run --output-format csv -- python3 bench.py --only k4 --k4-which $w
    step k4write$w 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $P/k4write$w -o run --output-format csv -- python3 bench.py --only k4 --k4-which $w
  done
  step mfma 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace -d $P/mfma -o run --output-format csv -- python3 bench.py --only dense_mfma
  python3 scripts/pmc_traffic.py $P/k4fetch2d $P/k4write2d "pds_dual_kernel" pds_dual_kernel@2048x2048 $P/traffic_k4.json $T || true
  python3 scripts/pmc_traffic.py $P/k4fetch3d $P/k4write3d "pds_dual_kernel" pds_dual_kernel@1024x1024x1024 $P/traffic_k4.json $T || true
  grep -h "" $O/small_weights.jsonl 2>/dev/null || true
fi
if [ "$S" = "ab1" ]; then
  step pdstests 600 $PT -m gpu tests/test_gpu_pds_fused.py tests/test_gpu_long_trajectories.py -k "pds or dual"
  step ntab 600 python3 scripts/nt_ab_probe.py 1024 2
  step gaptrace 300 rocprofv3 --kernel-trace -d $P/gap -o run --output-format csv -- python3 scripts/driver_gap_probe.py 20 5
  python3 scripts/driver_gap_probe.py 20 5 > /dev/null 2>&1 || true
  step k4fetch3d 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $P/k4fetch3d -o run --output-format csv -- python3 bench.py --only k4 --k4-which 3d
  step k4write3d 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $P/k4write3d -o run --output-format csv -- python3 bench.py --only k4 --k4-which 3d
  python3 scripts/pmc_traffic.py $P/k4fetch3d $P/k4write3d "pds_dual_kernel" pds_dual_kernel@1024x1024x1024 $P/traffic_k4.json $T || true
  B3="python3 bench.py --only c3 --c3-steps 3"
  step fetchc3 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $P/fetchc3 -o run --output-format csv -- $B3
  step writec3 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $P/writec3 -o run --output-format csv -- $B3
  python3 scripts/pmc_traffic.py $P/fetchc3 $P/writec3 "pds_march_kernel<float, 6, 1, true, false, true, true>" pds_march_kernel_pd3o@1024^3 $P/traffic_c3.json $T || true
  python3 scripts/pmc_traffic.py $P/fetchc3 $P/writec3 "pds_march_kernel<float, 6, 1, false, false, true, true>" pds_march_kernel_cv@1024^3 $P/traffic_c3.json $T || true
fi
if [ "$S" = "gap" ]; then
  step pgdtests 600 $PT -m gpu tests/test_gpu_pgd_variants.py tests/test_gpu_solver_engine.py tests/test_gpu_parity.py -k "pgd or relerr or speculative or async or trajectory"
  step drv1 120 $DRV
  step drv2 120 $DRV
  step drv3 120 $DRV
  step gaptrace 300 rocprofv3 --kernel-trace -d $P/gap -o run --output-format csv -- python3 scripts/driver_gap_probe.py 20 5
  grep -h '^\[{' $O/gaptrace.log > $O/stamps.json || true
  python3 scripts/driver_gap_probe.py --analyze $P/gap $O/stamps.json || true
fi
if [ "$S" = "c4prof" ]; then
  step k4wgs 300 python3 scripts/k4_wgs_probe.py 0,2048,8192
  step c4 300 python3 bench.py --only c4
  step c4trace 300 rocprofv3 --kernel-trace --stats -d $P/c4 -o run --output-format csv -- python3 bench.py --only c4
  python3 scripts/c4_timeline.py $P/c4 || true
fi
if [ "$S" = "c4b" ]; then
  step cgtests 600 $PT -m gpu tests/test_gpu_dense_normal.py tests/test_gpu_parity.py tests/test_gpu_distributed.py -k "cg or admm or normal or sharded or dense"
  step c4 300 python3 bench.py --only c4
  step c4trace 300 rocprofv3 --kernel-trace --stats -d $P/c4b -o run --output-format csv -- python3 bench.py --only c4
  python3 scripts/c4_timeline.py $P/c4b || true
  step c4host 300 python3 scripts/c4_host_prof.py
fi
if [ "$S" = "nab" ]; then
  step cgtests 600 $PT -m gpu tests/test_gpu_dense_normal.py tests/test_gpu_parity.py tests/test_gpu_bench_shapes.py tests/test_gpu_distributed.py -k "cg or admm or normal or sharded or dense"
  step nab 600 python3 scripts/normal_ab.py --all
  step c4 300 python3 bench.py --only c4
  step c4stamps 300 python3 scripts/c4_host_stamps.py
fi
if [ "$S" = "ngp" ]; then
  export PXA_LIB_PATH=build/libpyxu_amd_probe.so
  step ngp0 120 python3 scripts/normal_group_probe.py 0
  step ngp16 120 python3 scripts/normal_group_probe.py 16
  unset PXA_LIB_PATH
  step nab 600 python3 scripts/normal_ab.py --all
fi
if [ "$S" = "pgdp" ]; then
  export PXA_LIB_PATH=build/libpyxu_amd_probe.so
  step stag 300 python3 scripts/pgd_modes_probe.py stagger
  step modes 300 python3 scripts/pgd_modes_probe.py diag 2048
  for d in 0 64 128 192; do
    step pmc_lds_$d 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_WAVES -d $P/lds_$d -o run --output-format csv -- python3 scripts/pgd_modes_probe.py one $d
  done
  unset PXA_LIB_PATH
fi
if [ "$S" = "timer" ]; then
  for i in 1 2 3; do
    step drvt$i 120 $DRV
    step drvn$i 120 $DRV --no-kernel-timer
  done
fi
if [ "$S" = "fft3" ]; then
  step ffttests 600 $PT -m gpu tests/test_gpu_fft.py tests/test_gpu_stencil_fft.py
  step ffttrace 120 rocprofv3 --kernel-trace --stats -d $P/fft_trace -o run --output-format csv -- python3 scripts/fft_probe.py 2048x2048
  step ffttrace4 120 rocprofv3 --kernel-trace --stats -d $P/fft_trace4 -o run --output-format csv -- python3 scripts/fft_probe.py 4096x4096
  step ffttrace3 120 rocprofv3 --kernel-trace --stats -d $P/fft_trace3 -o run --output-format csv -- python3 scripts/fft_probe.py 256x256x256
fi
if [ "$S" = "fft2" ]; then
  step ffttests 600 $PT -m gpu tests/test_gpu_fft.py tests/test_gpu_stencil_fft.py
  step ops 300 python3 scripts/bench_ops.py
  step ffttrace 120 rocprofv3 --kernel-trace --stats -d $P/fft_trace -o run --output-format csv -- python3 scripts/fft_probe.py 2048x2048
  step fftfetch 90 rocprofv3 --pmc FETCH_SIZE -d $P/fft_fetch -o run --output-format csv -- python3 scripts/fft_probe.py 2048x2048 10
  step fftwrite 90 rocprofv3 --pmc WRITE_SIZE -d $P/fft_write -o run --output-format csv -- python3 scripts/fft_probe.py 2048x2048 10
  step fftsq 90 rocprofv3 --pmc SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_WAVES -d $P/fft_sq -o run --output-format csv -- python3 scripts/fft_probe.py 2048x2048 10
fi
if [ "$S" = "fft4" ]; then
  step ffttests 600 $PT -m gpu tests/test_gpu_fft.py tests/test_gpu_stencil_fft.py
  PXA_LIB_PATH=build/libpyxu_amd_probe.so step fftmodes 200 rocprofv3 --kernel-trace -d $P/fft_modes -o run --output-format csv -- python3 scripts/fft_modes_probe.py 2048x2048
  step fftfetch 90 rocprofv3 --pmc FETCH_SIZE -d $P/fft_fetch -o run --output-format csv -- python3 scripts/fft_probe.py 2048x2048 10
  step fftwrite 90 rocprofv3 --pmc WRITE_SIZE -d $P/fft_write -o run --output-format csv -- python3 scripts/fft_probe.py 2048x2048 10
  step fftsq 90 rocprofv3 --pmc SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_WAVES -d $P/fft_sq -o run --output-format csv -- python3 scripts/fft_probe.py 2048x2048 10
  step fftsq2 90 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES -d $P/fft_sq2 -o run --output-format csv -- python3 scripts/fft_probe.py 2048x2048 10
fi
if [ "$S" = "fft" ]; then
  step ops 300 python3 scripts/bench_ops.py
  step ffttrace 120 rocprofv3 --kernel-trace --stats -d $P/fft_trace -o run --output-format csv -- python3 scripts/fft_probe.py 2048x2048
  step fftfetch 90 rocprofv3 --pmc FETCH_SIZE -d $P/fft_fetch -o run --output-format csv -- python3 scripts/fft_probe.py 2048x2048 10
  step fftwrite 90 rocprofv3 --pmc WRITE_SIZE -d $P/fft_write -o run --output-format csv -- python3 scripts/fft_probe.py 2048x2048 10
  step fftsq 90 rocprofv3 --pmc SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_WAVES -d $P/fft_sq -o run --output-format csv -- python3 scripts/fft_probe.py 2048x2048 10
fi
if [ "$S" = "k4off" ]; then
  step k4off 300 python3 scripts/k4_offset_probe.py
fi
if [ "$S" = "pgdd" ]; then
  export PXA_LIB_PATH=build/libpyxu_amd_probe.so
  step modes 300 python3 scripts/pgd_modes_probe.py diag 2048 4096
fi
if [ "$S" = "ops" ]; then
  step ops 300 python3 scripts/bench_ops.py
fi
if [ "$S" = "grad" ]; then
  step gradtests 300 $PT -m gpu tests/test_gpu_gradient_kernels.py
  step gradab 300 python3 scripts/grad_ab.py
  step gradtrace 120 rocprofv3 --kernel-trace --stats -d $P/grad_trace -o run --output-format csv -- python3 scripts/grad_probe.py 1024x1024x1024
  step gradfetch 120 rocprofv3 --pmc FETCH_SIZE -d $P/grad_fetch -o run --output-format csv -- python3 scripts/grad_probe.py 1024x1024x1024 3
  step gradwrite 120 rocprofv3 --pmc WRITE_SIZE -d $P/grad_write -o run --output-format csv -- python3 scripts/grad_probe.py 1024x1024x1024 3
fi
if [ "$S" = "stnd" ]; then
  step stndtests 300 $PT -m gpu tests/test_gpu_stencil_nd_tile.py tests/test_gpu_stencil_fft.py tests/test_gpu_filters.py tests/test_gpu_gradient_kernels.py
  step ops 300 python3 scripts/bench_ops.py
fi
if [ "$S" = "f64" ]; then
  step f64a 120 python3 scripts/fft_f64_check.py 0
  step f64b 120 python3 scripts/fft_f64_check.py 1024
  step f64c 120 python3 scripts/fft_f64_check.py 256
  step f64d 120 python3 scripts/fft_f64_check.py 1
  step f64e 120 python3 scripts/fft_f64_check.py 0
fi
if [ "$S" = "full" ]; then
  step pytest 1000 $PT tests -m gpu
  step smoke 150 python -c "import __graft_entry__ as g; g.smoke()"
fi
if [ "$S" = "bench" ]; then
  step bench 1000 python bench.py --steps 20 --warmup 5
fi
echo done

# usage: bash scripts/gpu_r03.sh <tag> [quick|noprof|profonly]
# One GPU call of round 3: the PGD mode parity tests first, then the whole -m gpu suite, smoke, the
# default bench line (N=1, every sub-record), rocprofv3 kernel trace / stats of the headline, SQ counter
# passes and FETCH / WRITE traffic of pgd_tv2d_kernel at 2048^2, 4096^2 and C5, and of the look-ahead PDS
# step's kernels B and D at C3 1024^3.  Test failures
# (rc 1) do not stop the run; any other failure (fault, abort, timeout) ends it there.
set -o pipefail
T=${1:-r03}
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
if [ "$2" != "profonly" ]; then
step variants 300 $PT tests/test_gpu_pgd_variants.py -m gpu
[ "$2" = "quick" ] || step pytest 900 $PT tests -m gpu --ignore=tests/test_gpu_pgd_variants.py
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 600 python bench.py
fi
[ "$2" = "noprof" ] && { echo done; exit 0; }
P=$O/prof
mkdir -p $P
step trace 300 rocprofv3 --kernel-trace --stats -d $P/trace -o run --output-format csv -- python3 bench.py --no-sub --cpu-seconds 0 --steps 200 --warmup 20
B="python3 bench.py --no-sub --cpu-seconds 0 --steps 20 --warmup 5 --prime-seconds 0"
step sq1 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY --kernel-trace -d $P/sq1 -o run --output-format csv -- $B
step sq2 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_IDX_ACTIVE --kernel-trace -d $P/sq2 -o run --output-format csv -- $B
step fetch 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $P/fetch -o run --output-format csv -- $B
step write 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $P/write -o run --output-format csv -- $B
B4="python3 bench.py --only c2_4096 --c4096-steps 20"
step fetch4k 180 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $P/fetch4k -o run --output-format csv -- $B4
step write4k 180 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $P/write4k -o run --output-format csv -- $B4
B5="python3 bench.py --only c5 --c5-steps 10 --c5-warmup 2"
step fetchc5 180 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $P/fetchc5 -o run --output-format csv -- $B5
step writec5 180 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $P/writec5 -o run --output-format csv -- $B5
B3="python3 bench.py --only c3 --c3-steps 3"
step fetchc3 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $P/fetchc3 -o run --output-format csv -- $B3
step writec3 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $P/writec3 -o run --output-format csv -- $B3
step sqc3 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY --kernel-trace -d $P/sqc3 -o run --output-format csv -- $B3
python3 scripts/pmc_traffic.py $P/fetchc3 $P/writec3 "pds_march_kernel<float, 6, 1, true, false, true>" pds_march_kernel_pd3o@1024^3 $P/traffic.json $T
python3 scripts/pmc_traffic.py $P/fetchc3 $P/writec3 "pds_march_kernel<float, 6, 1, false, false, true>" pds_march_kernel_cv@1024^3 $P/traffic.json $T
python3 scripts/pmc_traffic.py $P/fetchc3 $P/writec3 "pds_plane_kernel<float, 6, 0>" pds_plane_kernel_pd3o@1024^3 $P/traffic.json $T
python3 scripts/pmc_traffic.py $P/fetchc3 $P/writec3 "pds_plane_kernel<float, 6, 2>" pds_plane_kernel_cv@1024^3 $P/traffic.json $T
K="pgd_tv2d_kernel<float, 6>"
python3 scripts/pmc_traffic.py $P/fetch $P/write "$K" pgd_tv2d_kernel@2048x2048 $P/traffic.json $T
python3 scripts/pmc_traffic.py $P/fetch4k $P/write4k "$K" pgd_tv2d_kernel@4096x4096 $P/traffic.json $T
python3 scripts/pmc_traffic.py $P/fetchc5 $P/writec5 "$K" pgd_tv2d_kernel@512x512x512 $P/traffic.json $T
for p in sq1 sq2 trace; do python3 scripts/pmc_summary.py $P/$p pgd_tv2d; done > $P/summary.txt
for k in "pds_march_kernel<float, 6, 1, true, false, true>" "pds_march_kernel<float, 6, 1, false, false, true>" \
         "pds_plane_kernel<float, 6, 0>" "pds_plane_kernel<float, 6, 2>"; do
  echo "-- C3 $k"; python3 scripts/pmc_summary.py $P/sqc3 "$k"; done >> $P/summary.txt
cat $P/summary.txt
echo done

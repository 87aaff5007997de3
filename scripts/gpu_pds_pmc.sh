# SQ counters + FETCH/WRITE of the PD3O / CondatVu kernels (512^3 to keep the passes short)
set -o pipefail
O=gpurun_out/${1:-pdspmc}
mkdir -p $O
export TMPDIR=/tmp PXA_N=512 PXA_STEPS=4 PXA_GENERIC_N=0
B="python3 scripts/bench_pds.py"
run() { local name=$1; shift; echo "== $name"; timeout -k 10 150 rocprofv3 "$@" --kernel-trace -d $O/$name -o run --output-format csv -- $B > $O/$name.log 2>&1; local rc=$?; echo "   rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
run sq1 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY
run sq2 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_IDX_ACTIVE
run fetch --pmc FETCH_SIZE
run write --pmc WRITE_SIZE
for p in sq1 sq2 fetch write; do for k in "pds_plane_kernel<float, 6, true>" "pds_plane_kernel<float, 6, false>" "pds_dual_kernel" "pds_axis0_kernel"; do echo "[$p] $k"; python3 scripts/pmc_summary.py $O/$p "$k"; done; done > $O/summary.txt
cat $O/summary.txt

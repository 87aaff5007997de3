# PMC passes of the fused PGD step alone (scripts/prof_pgd.py) -> gpurun_out/pmc_pgd/<pass>
set -o pipefail
D=gpurun_out/pmc_pgd
mkdir -p $D
export TMPDIR=/tmp
run() { name=$1; shift; timeout -s KILL 90 rocprofv3 "$@" -d $D/$name -o run --output-format csv -- python3 scripts/prof_pgd.py > $D/$name.log 2>&1; }
run trace --kernel-trace --stats \
 && run p1 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY --kernel-trace \
 && run p2 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_IDX_ACTIVE --kernel-trace \
 && run p3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_LEVEL_WAVES SQ_CYCLES SQ_BUSY_CU_CYCLES SQ_INSTS_SMEM SQ_LDS_UNALIGNED_STALL SQ_IFETCH --kernel-trace \
 && for p in p1 p2 p3; do python3 scripts/pmc_summary.py $D/$p pgd_tv2d; done > $D/summary.txt \
 && python3 scripts/pmc_summary.py $D/trace pgd_tv2d >> $D/summary.txt

# usage: bash scripts/gpu_prof.sh <outdir>   (kernel trace + PMC passes of the fused PGD step)
set -o pipefail
D=${1:-gpurun_out/prof}
mkdir -p $D
export TMPDIR=/tmp
run() { name=$1; shift; timeout -k 10 300 rocprofv3 "$@" -d $D/$name -o run --output-format csv -- python3 scripts/prof_pgd.py > $D/$name.log 2>&1; }
run trace --kernel-trace --stats \
 && run pmc1 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY --kernel-trace \
 && run pmc3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_IDX_ACTIVE --kernel-trace \
 && run pmc4 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace \
 && run pmc5 --pmc FETCH_SIZE WRITE_SIZE --kernel-trace \
 && echo ok

# usage: bash scripts/gpu_prof_occ.sh <outdir>  -- occupancy / instruction-fetch counters of the fused step
set -o pipefail
D=${1:-gpurun_out/profocc}
mkdir -p $D
export TMPDIR=/tmp
run() { name=$1; shift; timeout -k 10 300 rocprofv3 "$@" -d $D/$name -o run --output-format csv -- python3 scripts/prof_pgd.py > $D/$name.log 2>&1; }
run trace --kernel-trace --stats \
 && run o1 --pmc SQ_LEVEL_WAVES SQ_CYCLES SQ_BUSY_CU_CYCLES SQ_WAVES --kernel-trace \
 && run o2 --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_IFETCH SQ_WAVE_CYCLES --kernel-trace \
 && run o3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --kernel-trace \
 && run o4 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY --kernel-trace \
 && echo ok

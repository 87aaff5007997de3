# dynamic VALU instruction mix of the headline PGD kernel (two rocprofv3 PMC passes), bash scripts/pmc_pgd_valu.sh <tag>
set -o pipefail
T=${1:-r06w}
P=gpurun_out/$T/prof
mkdir -p $P
export TMPDIR=/tmp
DRV="python3 bench.py --steps 20 --warmup 5 --no-sub --cpu-seconds 0"
timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_INT64 --kernel-trace -d $P/valu1 -o run --output-format csv -- $DRV > gpurun_out/$T/valu1.log 2>&1 &&
timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_SALU SQ_INSTS_LDS_LOAD SQ_INSTS_LDS_STORE SQ_INSTS_BRANCH SQ_INSTS_VALU_FLOPS_FP32 --kernel-trace -d $P/valu2 -o run --output-format csv -- $DRV > gpurun_out/$T/valu2.log 2>&1 &&
python3 scripts/pmc_sum.py "pgd_tv2d_kernel<float, 6>" $P/valu1 $P/valu2 > gpurun_out/$T/valu_summary.txt 2>&1

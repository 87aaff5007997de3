set -o pipefail
mkdir -p gpurun_out/prof2
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof2/trace -o run --output-format csv -- python3 scripts/prof_pgd.py > gpurun_out/prof2/trace.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY --kernel-trace -d gpurun_out/prof2/pmc1 -o run --output-format csv -- python3 scripts/prof_pgd.py > gpurun_out/prof2/pmc1.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_IDX_ACTIVE --kernel-trace -d gpurun_out/prof2/pmc3 -o run --output-format csv -- python3 scripts/prof_pgd.py > gpurun_out/prof2/pmc3.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace -d gpurun_out/prof2/pmc4 -o run --output-format csv -- python3 scripts/prof_pgd.py > gpurun_out/prof2/pmc4.log 2>&1 || exit 1
echo ok

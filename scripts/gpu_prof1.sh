set -o pipefail
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/trace -o run --output-format csv -- python3 scripts/prof_pgd.py > gpurun_out/prof/trace.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY --kernel-trace -d gpurun_out/prof/pmc1 -o run --output-format csv -- python3 scripts/prof_pgd.py > gpurun_out/prof/pmc1.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/prof/pmc2 -o run --output-format csv -- python3 scripts/prof_pgd.py > gpurun_out/prof/pmc2.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD --kernel-trace -d gpurun_out/prof/pmc3 -o run --output-format csv -- python3 scripts/prof_pgd.py > gpurun_out/prof/pmc3.log 2>&1 || exit 1
find gpurun_out/prof -name "*.csv" | head -20

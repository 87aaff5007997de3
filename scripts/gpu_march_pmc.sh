# usage: bash scripts/gpu_march_pmc.sh <tag> -- bit-exactness debug, timing probes and SQ counters of the
# march kernel (PXA_TUNE_PGD_KERNEL = 5) beside the tile kernel
set -o pipefail
T=$1
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
(for s in "256 256" "2048 2048" "256 256 0.3" "1000 1004 2.0"; do timeout -k 10 60 python scripts/march_debug.py $s || exit 1; done) > $O/debug.txt 2>&1 || { cat $O/debug.txt; exit 1; }
cat $O/debug.txt
timeout -k 10 120 python scripts/pgd_probe.py base 0=5 0=5,3=1 0=5,3=2 n=4096 n=4096,0=5 n=4096,0=5,3=1 > $O/probe.txt 2>&1 || { cat $O/probe.txt; exit 1; }
cat $O/probe.txt
for k in 0 5; do
  timeout -s KILL 60 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY --kernel-trace -d $O/sq1_$k -o run --output-format csv -- python3 scripts/pgd_probe.py 0=$k > $O/sq1_$k.log 2>&1 || exit 1
  timeout -s KILL 60 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_IDX_ACTIVE --kernel-trace -d $O/sq2_$k -o run --output-format csv -- python3 scripts/pgd_probe.py 0=$k > $O/sq2_$k.log 2>&1 || exit 1
done
for k in 0 5; do echo "== kernel $k"; python3 scripts/pmc_summary.py $O/sq1_$k pgd_; python3 scripts/pmc_summary.py $O/sq2_$k pgd_; done
timeout -k 10 120 python scripts/pgd_probe.py 0=5,4=2 0=5,4=4 0=5,4=8 0=5,4=16 n=4096,0=5,4=8 n=4096,0=5,4=32 > $O/probe_sb.txt 2>&1 || { cat $O/probe_sb.txt; exit 1; }
cat $O/probe_sb.txt

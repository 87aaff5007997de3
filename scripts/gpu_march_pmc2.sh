# usage: bash scripts/gpu_march_pmc2.sh <tag> <probe-spec>... -- LDS counters of the march kernel per probe spec
set -o pipefail
T=$1; shift
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
for c in "$@"; do
  d=$O/$(echo $c | tr ',=.' '_-p')
  timeout -s KILL 60 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES --kernel-trace --stats -d $d -o run --output-format csv -- python3 scripts/pgd_probe.py $c > $d.log 2>&1 || { tail -5 $d.log; exit 1; }
  echo "== $c"; python3 scripts/pmc_summary.py $d pgd_
done

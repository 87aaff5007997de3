# usage: bash scripts/pgd_probe.sh <tag> <config>... -- rocprofv3 average duration of pgd_tv2d_kernel per probe config
set -o pipefail
T=$1; shift
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
for c in "$@"; do
  d=$O/$(echo $c | tr ',=.' '_-p')
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $d -o run --output-format csv -- python3 scripts/pgd_probe.py $c > $d.log 2>&1 || { echo "$c failed rc=$?"; tail -5 $d.log; exit 1; }
  f=$(find $d -name 'run_kernel_stats.csv' | head -1)
  avg=$(python3 -c "import csv,sys; print([r['AverageNs'] for r in csv.DictReader(open('$f')) if 'pgd_tv2d' in r['Name']][0])")
  echo "$c avg_ns=$avg"
done

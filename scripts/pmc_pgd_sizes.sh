# FETCH / WRITE PMC passes of the PGD tile kernel at 4096^2 (c2_4096) and C5 (512 x 512^2), one pass per
# counter, into profiles-ready traffic entries (scripts/pmc_traffic.py).
export TMPDIR=/tmp; T=${1:-r05zm}; P=gpurun_out/$T/prof; mkdir -p $P
set -o pipefail
for cfg in c2_4096 c5; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --pmc $c --kernel-trace -d $P/${cfg}_$c -o run --output-format csv -- python3 bench.py --only $cfg > gpurun_out/$T/${cfg}_$c.log 2>&1 || exit 1
  done
done
python3 scripts/pmc_traffic.py $P/c2_4096_FETCH_SIZE $P/c2_4096_WRITE_SIZE pgd_tv2d_kernel pgd_tv2d_kernel@4096x4096 $P/traffic_sizes.json $T
python3 scripts/pmc_traffic.py $P/c5_FETCH_SIZE $P/c5_WRITE_SIZE pgd_tv2d_kernel pgd_tv2d_kernel@512x512x512 $P/traffic_sizes.json $T
cat $P/traffic_sizes.json

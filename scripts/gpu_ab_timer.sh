set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
timeout -k 10 120 python bench.py --cpu-seconds 0 --no-kernel-timer > gpurun_out/ab_off_$i.log 2>&1 && tail -1 gpurun_out/ab_off_$i.log | cut -c1-200 || exit 1
timeout -k 10 120 python bench.py --cpu-seconds 0 > gpurun_out/ab_on_$i.log 2>&1 && tail -1 gpurun_out/ab_on_$i.log | cut -c1-200 || exit 1
done

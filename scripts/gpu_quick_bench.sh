# quick bench sweep: default workload + a small image (host-overhead floor of the solver step)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 python bench.py --cpu-seconds 0 > gpurun_out/qb_2048.log 2>&1 && tail -1 gpurun_out/qb_2048.log | cut -c1-220 \
 && timeout -k 10 120 python bench.py --cpu-seconds 0 --n 64 > gpurun_out/qb_64.log 2>&1 && tail -1 gpurun_out/qb_64.log | cut -c1-220 \
 && timeout -k 10 120 python bench.py --cpu-seconds 0 --n 64 --stop-rate 1 > gpurun_out/qb_64s1.log 2>&1 && tail -1 gpurun_out/qb_64s1.log | cut -c1-220

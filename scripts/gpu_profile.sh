# usage: bash scripts/gpu_profile.sh <tag>  -- rocprofv3 kernel-trace/stats of the bench command + PMC traffic
# passes (FETCH_SIZE and WRITE_SIZE in separate runs) of the dominant kernel.  Results: gpurun_out/prof_<tag>/
set -o pipefail
T=${1:-r01}
D=gpurun_out/prof_$T
mkdir -p $D
export TMPDIR=/tmp
CMD="python3 bench.py --steps 200 --warmup 20 --cpu-seconds 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/trace -o run --output-format csv -- $CMD > $D/trace.log 2>&1 \
 && timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $D/fetch -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --cpu-seconds 0 > $D/fetch.log 2>&1 \
 && timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $D/write -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --cpu-seconds 0 > $D/write.log 2>&1 \
 && python3 scripts/pmc_traffic.py $D/fetch $D/write pgd_tv2d_kernel pgd_tv2d_kernel@2048x2048 $D/traffic.json \
 && tail -1 $D/trace.log

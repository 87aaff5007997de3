# usage: bash scripts/gpu_pc2.sh <tag>: pipelined PGD kernel phase traces with producers / consumers idled
set -o pipefail
O=gpurun_out/${1:-pc2}
mkdir -p $O
for d in 0 64 128; do
  timeout -k 10 120 python -u scripts/pc_trace.py 2048 $d 2>&1 | tee -a $O/trace.log || exit $?
done

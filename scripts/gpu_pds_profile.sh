# usage: bash scripts/gpu_pds_profile.sh <tag> -- C3 (1024^3 PD3O / Condat-Vu) kernel trace + per-kernel
# FETCH_SIZE / WRITE_SIZE passes.  Results: gpurun_out/pdsprof_<tag>/
set -o pipefail
T=${1:-r01}
D=gpurun_out/pdsprof_$T
mkdir -p $D
export TMPDIR=/tmp
export PXA_N=${PXA_N:-1024} PXA_GENERIC_N=0
PXA_STEPS=10 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/trace -o run --output-format csv -- python3 scripts/bench_pds.py > $D/trace.log 2>&1 \
 && PXA_STEPS=3 timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $D/fetch -o run --output-format csv -- python3 scripts/bench_pds.py > $D/fetch.log 2>&1 \
 && PXA_STEPS=3 timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $D/write -o run --output-format csv -- python3 scripts/bench_pds.py > $D/write.log 2>&1 \
 && grep -v amdgpu.ids $D/trace.log | tail -4

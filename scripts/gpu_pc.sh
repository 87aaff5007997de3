# usage: bash scripts/gpu_pc.sh <tag>: PGD kernel-variant parity tests, then the tile / pipelined A/B probe.
set -o pipefail
T=${1:-pc}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_gpu_pgd_variants.py -m gpu > $O/variants.log 2>&1
rc=$?; echo "variants rc=$rc"; tail -15 $O/variants.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u scripts/pgd_modes_probe.py 2048 4096 512:512 2>&1 | tee $O/probe.log
timeout -k 10 120 python -u scripts/pc_trace.py 2048 2>&1 | tee $O/trace2048.log
timeout -k 10 120 python -u scripts/pc_trace.py 512:512 2>&1 | tee $O/trace_c5.log

# usage: bash scripts/gpu_quick3.sh <tag>: whole -m gpu suite, host-cost probe, headline bench line (no c3)
set -o pipefail
O=gpurun_out/${1:-q3}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests -m gpu > $O/pytest.log 2>&1
rc=$?; tail -5 $O/pytest.log; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u scripts/host_cost_sr1.py 128 > $O/hostcost.log 2>&1 || exit $?
tail -4 $O/hostcost.log
timeout -k 10 400 python -u bench.py --c3-n 0 --cpu-seconds 0 > $O/bench.log 2>&1 || exit $?
tail -1 $O/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['roofline']['kernel_ms'], d['stop_rate_1'], d['c5']['value'], d['c5']['roofline']['kernel_ms'], d['c4']['ms_per_cg_iter'], d['c2_4096']['roofline']['kernel_ms'])"

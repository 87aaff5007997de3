# stop_rate=1 A/B: speculative stop checks on (default) vs off (PXA_NO_SPEC=1); C4 ADMM line
set -o pipefail
O=gpurun_out/sr1
mkdir -p $O
for v in 0 1 0 1; do
  PXA_NO_SPEC=$v timeout -k 10 120 python bench.py --no-sub --cpu-seconds 0 --stop-rate 1 > $O/b$v.log 2>&1 || exit 1
  python -c "import json; d=json.loads(open('$O/b$v.log').read().strip().splitlines()[-1]); print('nospec=$v', d['value'], d['ms_per_step'])"
done
PXA_NO_SPEC=0 timeout -k 10 120 python bench.py --no-sub --cpu-seconds 0 > $O/b50.log 2>&1 && python -c "import json; d=json.loads(open('$O/b50.log').read().strip().splitlines()[-1]); print('sr50', d['value'], d['ms_per_step'])"
timeout -k 10 300 python -u scripts/bench_admm.py > $O/admm.log 2>&1; tail -1 $O/admm.log

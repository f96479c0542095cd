#!/bin/bash
# round 3: per-role k_chain kernels + one-launch individual Miller loops -- tests, bench at 14 / 16 contexts, sub-records
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3i
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
B="python -u bench.py --steps 8 --warmup 1 --no-cpu-baseline --no-sub-records --latency-runs 10"
for cfg in "14 8" "16 8"; do
  set -- $cfg
  n=r_${1}x${2}
  timeout -k 10 240 $B --inflight $1 --calls-per-pass $2 > $O/$n.json 2> $O/$n.err || { echo "$n failed"; tail $O/$n.err; exit 1; }
  echo "$n $(python3 -c "import json;d=json.load(open('$O/$n.json'));print(d['value'],d['ms_per_step'],d['p50_latency_ms_128'])")"
done
timeout -k 10 400 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --latency-runs 3 > $O/sub.json 2> $O/sub.err || { echo "sub failed"; tail $O/sub.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/sub.json'));print({k:(d[k].get('sets_per_s'),d[k].get('p50_ms')) for k in ('cfg3','cfg4_slice','cfg4_slice_batchable')})"
echo done

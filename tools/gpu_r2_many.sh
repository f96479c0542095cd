#!/bin/bash
# verify_many: the new parity test, then throughput vs (contexts, calls per pass) with
# 1024-set calls (gpurun_out/many).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/many
mkdir -p $O; cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v -k "verify_many or cfg2_1024" --timeout 100 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Timeout|Error|assert" $O/pytest.log | tail -30; exit 1; }
tail -1 $O/pytest.log
for cfg in ${MANY_CFGS:-"20 1" "10 2" "8 4" "6 4" "4 8" "12 2" "16 2"}; do
  set -- $cfg
  tag=i$1_k$2
  timeout -k 10 300 python -u bench.py --inflight $1 --calls-per-pass $2 --steps ${STEPS:-10} --warmup 2 --latency-runs 2 --no-cpu-baseline > $O/$tag.json 2> $O/$tag.err || { echo "fail $tag"; tail -5 $O/$tag.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/$tag.json'));print('$tag', round(d['value']), d['ms_per_step'], d['stage_ms'])"
done

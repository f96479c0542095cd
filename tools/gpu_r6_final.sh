#!/bin/bash
# Round-6 final check on the GPU box: the GPU tests, smoke(), the default bench line
# (sub-records and CPU baseline included) and the N-API lines; each step has its own
# time limit and the script stops at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r6final}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 1100 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench.json'));print(d['value'],d['ms_per_step'],d['p50_latency_ms_128'])"
if [ -n "$NAPI" ]; then
  timeout -k 10 600 python -u bench.py --mode napi > $O/napi.json 2> $O/napi.err || { echo "napi bench failed"; tail -20 $O/napi.err; exit 1; }
  head -c 600 $O/napi.json; echo
fi
echo done

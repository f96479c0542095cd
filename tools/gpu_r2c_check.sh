#!/bin/bash
# Re-check after a rebuild: GPU parity suite, smoke, one driver-shaped bench line.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/chk
mkdir -p $O; cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Timeout|Error|assert" $O/pytest_gpu.log | tail -30; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --cpu-seconds 5 > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench.json'));print(round(d['value']), d['ms_per_step'], d['p50_latency_ms_128'], d['roofline']['frac'], d.get('cpu_baseline',{}).get('value'))"

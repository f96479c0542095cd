#!/bin/bash
# parity tests (-m gpu), then the default cfg2 bench line (driver shape: 20 steps)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/check
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "PASS|FAIL|Error|error" $O/pytest_gpu.log | tail -40; exit 1; }
grep -c PASSED $O/pytest_gpu.log; tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --latency-runs 5 > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench.json'));print(d['value'], d['p50_latency_ms_128'], d['stage_ms'])"

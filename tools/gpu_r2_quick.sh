#!/bin/bash
# parity tests, the cfg2 bench line and the N-API mode (gpurun_out/quick)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/quick
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error" $O/pytest_gpu.log | tail -30; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench.json'));print('cfg2', d['value'], d['p50_latency_ms_128'], d['roofline']['frac'], d['stage_ms'])"
timeout -k 10 300 python -u bench.py --mode napi --steps 8 --warmup 1 > $O/bench_napi.json 2> $O/bench_napi.err || { echo "napi bench failed"; tail -20 $O/bench_napi.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_napi.json'));print('napi', d['value'], d['napi'])"

#!/bin/bash
# Round-end evidence: GPU parity, the default bench line, and rocprofv3 kernel traces of
# the default bench and of a solo (1 batch in flight) run, whose k_psetn average is the
# launch time the roofline's solo HIP-event measurement should agree with.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 400 python -u bench.py > gpurun_out/bench_final.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/bench_final.log; exit 1; }
tail -1 gpurun_out/bench_final.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof/trace" -o bench --output-format csv -- python3 "$R/bench.py" --no-cpu-baseline > gpurun_out/prof/trace.log 2>&1 || { echo "trace failed"; tail -20 gpurun_out/prof/trace.log; exit 1; }
tail -1 gpurun_out/prof/trace.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof/solo" -o bench --output-format csv -- python3 "$R/bench.py" --no-cpu-baseline --inflight 1 --steps 8 --latency-runs 2 > gpurun_out/prof/solo.log 2>&1 || { echo "solo trace failed"; tail -20 gpurun_out/prof/solo.log; exit 1; }
tail -1 gpurun_out/prof/solo.log

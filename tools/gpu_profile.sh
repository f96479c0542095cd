#!/bin/bash
# Round-end evidence: GPU parity tests, the default bench line, a rocprofv3 kernel
# trace of the same bench command, and two PMC passes (HBM fetch / write bytes).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 400 python -u bench.py > gpurun_out/bench_full.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/bench_full.log; exit 1; }
tail -1 gpurun_out/bench_full.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof/trace" -o bench --output-format csv -- python3 "$R/bench.py" --no-cpu-baseline > gpurun_out/prof/trace.log 2>&1 || { echo "trace failed"; tail -20 gpurun_out/prof/trace.log; exit 1; }
tail -1 gpurun_out/prof/trace.log
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d "$R/gpurun_out/prof/pmc_fetch" -o bench --output-format csv -- python3 "$R/bench.py" --no-cpu-baseline --steps 3 --warmup 1 --inflight 1 --latency-runs 1 > gpurun_out/prof/pmc_fetch.log 2>&1 || { echo "pmc fetch failed"; tail -20 gpurun_out/prof/pmc_fetch.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d "$R/gpurun_out/prof/pmc_write" -o bench --output-format csv -- python3 "$R/bench.py" --no-cpu-baseline --steps 3 --warmup 1 --inflight 1 --latency-runs 1 > gpurun_out/prof/pmc_write.log 2>&1 || { echo "pmc write failed"; tail -20 gpurun_out/prof/pmc_write.log; exit 1; }
python tools/pmc_traffic.py gpurun_out/prof/pmc_fetch/bench_counter_collection.csv gpurun_out/prof/pmc_write/bench_counter_collection.csv gpurun_out/prof/pmc_traffic.json
find gpurun_out/prof -name "*.csv" | sort

#!/bin/bash
# GPU parity tests, then cfg2 with and without the merged check, and the cfg5 shape.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bench_cfg2.log 2>&1 || { echo "bench cfg2 failed"; tail -20 gpurun_out/bench_cfg2.log; exit 1; }
tail -1 gpurun_out/bench_cfg2.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-merged-check > gpurun_out/bench_cfg2_nomerge.log 2>&1 || { echo "bench nomerge failed"; tail -20 gpurun_out/bench_cfg2_nomerge.log; exit 1; }
tail -1 gpurun_out/bench_cfg2_nomerge.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline --roots 2 > gpurun_out/bench_cfg5.log 2>&1 || { echo "bench cfg5 failed"; tail -20 gpurun_out/bench_cfg5.log; exit 1; }
tail -1 gpurun_out/bench_cfg5.log

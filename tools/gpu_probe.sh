#!/bin/bash
# One GPU call: parity tests, Fp-product and cooperative-program probes, short bench.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 120 python -u tools/fpm_probe.py > gpurun_out/fpm_probe.log 2>&1 || { echo "fpm probe failed"; cat gpurun_out/fpm_probe.log; exit 1; }
cat gpurun_out/fpm_probe.log
timeout -k 10 300 python -u tools/coop_probe.py > gpurun_out/coop_probe.log 2>&1 || { echo "probe failed"; cat gpurun_out/coop_probe.log; exit 1; }
timeout -k 10 400 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/bench.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log

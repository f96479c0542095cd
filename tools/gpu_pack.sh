#!/bin/bash
# GPU parity suite with the default kernel choice and with every batch forced through
# the packed kernels (BLS_PACK=3, BLS_PACK=2), then the bench.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
for S in 3 2; do
BLS_PACK=$S timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_verifier.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu_pack$S.log 2>&1 || { echo "pytest (packed $S) failed"; tail -40 gpurun_out/pytest_gpu_pack$S.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_pack$S.log
done
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bench.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log

#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_napi.py -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/napi.log 2>&1; tail -40 gpurun_out/napi.log

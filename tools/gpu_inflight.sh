#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/inflight_probe.py > gpurun_out/inflight.log 2>&1 || { tail -20 gpurun_out/inflight.log; exit 1; }
cat gpurun_out/inflight.log

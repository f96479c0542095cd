#!/bin/bash
# The cfg5 slice's failing passes on the GPU box: tools/cfg5_probe.py plain (both jobs),
# then the job with invalid sets and the all-valid job each under a kernel trace.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r5c5}; mkdir -p $O
[ -n "$NOPROBE" ] || timeout -k 10 300 python -u tools/cfg5_probe.py ${ARGS} > $O/probe.json 2> $O/probe.err || { echo "probe failed"; tail -20 $O/probe.err; exit 1; }
[ -n "$NOPROBE" ] || grep -v "^\[" $O/probe.err | tail -3
# (the profiler starts the HIP runtime before the probe could set the queue count)
export GPU_MAX_HW_QUEUES=24
for run in ${RUNS:-invalid valid}; do
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/trace_$run -o run --output-format csv -- python3 $R/tools/cfg5_probe.py ${ARGS} --runs $run > $R/$O/trace_$run.log 2>&1) || { tail -20 $O/trace_$run.log; exit 1; }
done
echo done

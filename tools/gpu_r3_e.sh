#!/bin/bash
# round 3: GLV scalars + split SIMT Miller loops + k_chain roles out of line -- tests, in-flight sweep, sub-records, solo trace
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3e
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
B="python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-sub-records"
run() { local name=$1; shift; local envs=$1; shift; env $envs timeout -k 10 300 $B "$@" > $O/$name.json 2> $O/$name.err || { echo "$name failed"; tail $O/$name.err; exit 1; }; }
run split_10x8 BLS_ML_SIMT=2
run split_14x8 BLS_ML_SIMT=2 --inflight 14
run split_10x12 BLS_ML_SIMT=2 --calls-per-pass 12
run split_12x12 BLS_ML_SIMT=2 --inflight 12 --calls-per-pass 12
run coop_12x8 BLS_ML_SIMT=0 --inflight 12
timeout -k 10 400 python -u bench.py --steps 4 --warmup 1 --cpu-seconds 5 > $O/sub.json 2> $O/sub.err || { echo "sub failed"; tail $O/sub.err; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$O/prof" -o solo -- python3 "$GRAFT_REPO_ROOT/bench.py" --sets 8192 --inflight 1 --calls-per-pass 1 --steps 3 --warmup 1 --no-cpu-baseline --no-sub-records --latency-runs 3 > "$GRAFT_REPO_ROOT/$O/solo.json" 2> "$GRAFT_REPO_ROOT/$O/solo.err" || { echo "rocprof failed"; exit 1; }
echo done

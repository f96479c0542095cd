#!/bin/bash
# round 3: Miller-loop variants (split SIMT lines + f, fused SIMT, cooperative) on the bench, then a solo trace
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3d
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
B="python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-sub-records"
run() { local name=$1; shift; env "$@" timeout -k 10 300 $B > $O/$name.json 2> $O/$name.err || { echo "$name failed"; tail $O/$name.err; exit 1; }; }
run split_10x8 BLS_ML_SIMT=2
run fused_10x8 BLS_ML_SIMT=1
run coop_10x8 BLS_ML_SIMT=0
run split_q1_10x8 BLS_ML_SIMT=2 BLS_MLQ_WAVES=1
BLS_ML_SIMT=2 timeout -k 10 300 $B --inflight 14 > $O/split_14x8.json 2> $O/split_14x8.err || { echo "split14 failed"; tail $O/split_14x8.err; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$O/prof" -o solo -- python3 "$GRAFT_REPO_ROOT/bench.py" --sets 8192 --inflight 1 --calls-per-pass 1 --steps 3 --warmup 1 --no-cpu-baseline --no-sub-records --latency-runs 3 > "$GRAFT_REPO_ROOT/$O/solo.json" 2> "$GRAFT_REPO_ROOT/$O/solo.err" || { echo "rocprof failed"; exit 1; }
echo done

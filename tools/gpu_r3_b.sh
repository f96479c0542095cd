#!/bin/bash
# round 3: SIMT Miller loops -- GPU tests, bench with the cfg3 / cfg4 sub-records, solo trace
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3b
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-sub-records > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail $O/bench.err; exit 1; }
BLS_ML_SIMT=0 timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-sub-records > $O/bench_coop.json 2> $O/bench_coop.err || { echo "bench coop failed"; tail $O/bench_coop.err; exit 1; }
timeout -k 10 400 python -u bench.py --steps 4 --warmup 1 --cpu-seconds 5 > $O/bench_sub.json 2> $O/bench_sub.err || { echo "bench sub failed"; tail -20 $O/bench_sub.err; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$O/prof" -o solo -- python3 "$GRAFT_REPO_ROOT/bench.py" --sets 8192 --inflight 1 --calls-per-pass 1 --steps 3 --warmup 1 --no-cpu-baseline --no-sub-records --latency-runs 3 > "$GRAFT_REPO_ROOT/$O/solo.json" 2> "$GRAFT_REPO_ROOT/$O/solo.err" || { echo "rocprof failed"; exit 1; }
echo done

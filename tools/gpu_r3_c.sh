#!/bin/bash
# round 3: SIMT Miller loops + wavefront pubkey aggregation -- tests (incl. cfg4/cfg5 slices), bench variants
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3c
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
B="python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-sub-records"
timeout -k 10 300 $B > $O/b_w1_10x8.json 2> $O/err1 || { echo "bench1 failed"; tail $O/err1; exit 1; }
BLS_MLS_WAVES=2 timeout -k 10 300 $B > $O/b_w2_10x8.json 2> $O/err2 || { echo "bench2 failed"; tail $O/err2; exit 1; }
timeout -k 10 300 $B --inflight 16 > $O/b_w1_16x8.json 2> $O/err3 || { echo "bench3 failed"; tail $O/err3; exit 1; }
BLS_MLS_WAVES=2 timeout -k 10 300 $B --inflight 16 > $O/b_w2_16x8.json 2> $O/err4 || { echo "bench4 failed"; tail $O/err4; exit 1; }
BLS_ML_SIMT=0 timeout -k 10 300 $B --inflight 16 > $O/b_coop_16x8.json 2> $O/err5 || { echo "bench5 failed"; tail $O/err5; exit 1; }
timeout -k 10 400 python -u bench.py --steps 4 --warmup 1 --no-cpu-baseline > $O/b_sub.json 2> $O/err6 || { echo "bench sub failed"; tail -20 $O/err6; exit 1; }

# whole-run SIMD utilisation: VALU-active and wave cycles summed over every kernel of a short bench
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE -d "$GRAFT_REPO_ROOT/$O/pmc_util" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --no-sub-records --latency-runs 2 > "$GRAFT_REPO_ROOT/$O/pmc_util.log" 2>&1 || { echo "pmc failed"; tail "$GRAFT_REPO_ROOT/$O/pmc_util.log"; exit 1; }
echo pmc done

#!/bin/bash
# Round-6 A/B step on the GPU box (first used for the f side's lane-pair variant,
# profiles/r06_ab_mlf_pair4.json; then the timed-region shapes, r06_knee.json): GPU tests
# (TESTK filter), cfg2 lines at the CFGS shapes for each ENVS label (alternated), and a
# kernel trace of the 12 x 22 shape per TRACE label.
# Each step has its own time limit; the script stops at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r6mlf}
R=$GRAFT_REPO_ROOT
mkdir -p $O
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread ${TESTK:+-k "$TESTK"} > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
  tail -1 $O/pytest.log
fi
B="python -u bench.py --steps ${STEPS:-8} --warmup 2 --no-cpu-baseline --no-sub-records --latency-runs 10"
for ab in $(echo "${ENVS:-base:}" | tr ';' ' '); do
  label=${ab%%:*}; vars=$(echo "${ab#*:}" | tr ',' ' ')
  for cfg in ${CFGS}; do
    c=${cfg%x*}; k=${cfg#*x}
    n=${label}_${c}x${k}
    env $vars timeout -k 10 240 $B --inflight $c --calls-per-pass $k > $O/$n.json 2> $O/$n.err || { echo "$n failed"; tail -3 $O/$n.err; exit 1; }
    echo "$n $(python3 -c "import json;d=json.load(open('$O/$n.json'));print(d['value'],d['ms_per_step'],d['p50_latency_ms_128'])")"
  done
done
for ab in $(echo "${TRACE}" | tr ';' ' '); do
  label=${ab%%:*}; vars=$(echo "${ab#*:}" | tr ',' ' ')
  PB="python3 $R/bench.py --probe-only --inflight 12 --calls-per-pass 22 --steps 1 --warmup 0"
  (cd /tmp && export TMPDIR=/tmp && env $vars timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/$O/trace_$label -o run --output-format csv -- $PB > $R/$O/trace_$label.log 2>&1) || { tail -20 $O/trace_$label.log; exit 1; }
  python3 -c "
import csv,glob
f=glob.glob('$O/trace_$label/**/*kernel_stats.csv',recursive=True)[0]
for r in csv.DictReader(open(f)):
  n=r['Name'].split('(')[0].replace('void ','')
  if n.startswith(('k_ml','k_chain','k_pre','k_msm_seg')): print('$label', n, r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us')"
done
echo done

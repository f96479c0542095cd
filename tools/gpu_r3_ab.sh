#!/bin/bash
# round 3 measurement step: $TAG names the output dir; $TESTS=1 runs the GPU tests first;
# bench lines for $CFGS ("contexts calls" pairs); $PMC=1 adds SQ / HBM counter passes and a
# kernel trace over exactly one 32-call pass (--probe-only).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-ab}
mkdir -p $O
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
  tail -1 $O/pytest.log
fi
B="python -u bench.py --steps ${STEPS:-8} --warmup 1 --no-cpu-baseline --no-sub-records --latency-runs 10"
# CFGS: "16x8 12x12" (contexts x calls per pass); ENVS: env assignments applied to every line,
# each A/B label separated by ";" as "label:VAR=v,VAR2=w" ("base:" = no extra variables)
for ab in $(echo "${ENVS:-base:}" | tr ';' ' '); do
 label=${ab%%:*}; vars=$(echo "${ab#*:}" | tr ',' ' ')
 for cfg in ${CFGS:-16x8}; do
  c=${cfg%x*}; k=${cfg#*x}
  n=${label}_${c}x${k}
  env $vars timeout -k 10 240 $B --inflight $c --calls-per-pass $k > $O/$n.json 2> $O/$n.err || { echo "$n failed"; tail -3 $O/$n.err; exit 1; }
  echo "$n $(python3 -c "import json;d=json.load(open('$O/$n.json'));print(d['value'],d['ms_per_step'],d['p50_latency_ms_128'])")"
 done
done
if [ -n "$SUB" ]; then
  timeout -k 10 400 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --latency-runs 3 --inflight 16 > $O/sub.json 2> $O/sub.err || { echo "sub failed"; tail $O/sub.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/sub.json'));print(d['value'], {k:(d[k].get('sets_per_s'),d[k].get('p50_ms')) for k in ('cfg3','cfg4_slice','cfg4_slice_batchable')})"
fi
if [ -n "$PMC" ]; then
  cd /tmp && export TMPDIR=/tmp
  R=$GRAFT_REPO_ROOT
  P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_LDS"
  P2="SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH"
  P3="GRBM_GUI_ACTIVE GRBM_COUNT"
  P4="FETCH_SIZE"
  P5="WRITE_SIZE"
  # the probe pass runs the timed region's shape (one pass alone would pick the low-in-flight
  # one): $PMC_ENV, default the Pippenger sum and four items per k_mlf lane
  export ${PMC_ENV:-BLS_MSM=1 BLS_MLF_PER_LANE=4}
  PB="python3 $R/bench.py --probe-only --inflight 1 --calls-per-pass 32 --steps 1 --warmup 0"
  k=0
  for P in "$P1" "$P2" "$P3" "$P4" "$P5"; do
    k=$((k+1))
    timeout -s KILL 150 rocprofv3 --pmc $P -d $R/$O/pmc$k -o run --output-format csv -- $PB > $R/$O/pmc$k.log 2>&1 || { tail -20 $R/$O/pmc$k.log; exit 1; }
  done
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/$O/trace -o run --output-format csv -- $PB > $R/$O/trace.log 2>&1 || { tail -20 $R/$O/trace.log; exit 1; }
  cd $R
  python3 tools/pmc_summary.py $O/pmc_summary.json "exactly one pass of 32 cfg2 calls (32768 sets; bench.py --probe-only --inflight 1 --calls-per-pass 32 --steps 1 --warmup 0); setup kernels (k_sign, k_sk_to_pk, k_load_pubkeys, k_aggregate) are input synthesis" $O/pmc1 $O/pmc2 $O/pmc3 $O/pmc4 $O/pmc5 > $O/pmc_summary.txt
fi
echo done

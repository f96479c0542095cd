#!/bin/bash
# Round-4 measurement step on the GPU box.  $TAG names gpurun_out/<TAG>; each step has
# its own time limit and the script stops at the first failure.
#   TESTS=1   the GPU tests (pytest -m gpu)
#   BENCH=1   the default bench line (what the driver runs), gpurun_out/<TAG>/bench.json
#   CFGS="12x22 4x16"  cfg2 lines at contexts x calls per pass (ENVS as in gpu_r3_ab.sh)
#   SWEEP4=1  tools/sweep_cfg4.py (the cfg4 slice's knee)
#   PMC=1     SQ / HBM counter passes + a kernel trace of the timed region's shape:
#             --inflight $PMC_CTX (16) --calls-per-pass $PMC_CPP (22), one step, no warm-up
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r4}
mkdir -p $O
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread ${TESTK:+-k "$TESTK"} > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
  tail -1 $O/pytest.log
fi
if [ -n "$BENCH" ]; then
  timeout -k 10 600 python -u bench.py ${BENCH_ARGS:---steps 20 --warmup 5} > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
  python3 -c "
import json;d=json.load(open('$O/bench.json'))
print('bench', d['value'], d['ms_per_step'], d.get('p50_latency_ms_128'), d['roofline']['frac'])
print({k:(d[k].get('sets_per_s'),d[k].get('p50_ms')) for k in ('cfg3','cfg4_slice','cfg4_slice_batchable','cfg5_slice') if k in d})"
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
if [ -n "$SWEEP4" ]; then
  timeout -k 10 600 python -u tools/sweep_cfg4.py ${SWEEP4_ARGS} > $O/sweep_cfg4.json 2> $O/sweep_cfg4.err || { echo "sweep failed"; tail -5 $O/sweep_cfg4.err; exit 1; }
  cat $O/sweep_cfg4.err | grep -v "^\[" | tail -20
fi
if [ -n "$LAT" ]; then
  # the 128-set call (p50_latency_ms_128) under a kernel trace: per-kernel durations
  R=$GRAFT_REPO_ROOT
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/$O/lat -o run --output-format csv -- python3 $R/tools/lat_probe.py --runs 10 > $R/$O/lat.log 2>&1) || { tail -20 $O/lat.log; exit 1; }
  grep p50_ms $O/lat.log | tail -1
fi
if [ -n "$COOP" ]; then
  timeout -k 10 240 python -u tools/coop_probe.py > $O/coop_probe.json 2> $O/coop_probe.err || { echo "coop probe failed"; tail -5 $O/coop_probe.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/coop_probe.json'));[print(k,v) for k,v in d.items()]"
fi
if [ -n "$REHEARSE" ]; then
  # bench.py --gpus 2 with both ranks on this box's one GPU (launcher, gloo control
  # collectives, rank-0 line): cfg2 and the cfg4 job mode
  export BLS_BENCH_SHARE_DEVICE=1
  timeout -k 10 300 python -u bench.py --gpus 2 --inflight 4 --calls-per-pass 8 --steps 3 --warmup 1 --no-cpu-baseline --no-sub-records > $O/rehearse_cfg2.json 2> $O/rehearse_cfg2.err || { echo "rehearse cfg2 failed"; tail -20 $O/rehearse_cfg2.err; exit 1; }
  timeout -k 10 300 python -u bench.py --gpus 2 --mode cfg4 --inflight 4 --steps 2 --warmup 1 > $O/rehearse_cfg4.json 2> $O/rehearse_cfg4.err || { echo "rehearse cfg4 failed"; tail -20 $O/rehearse_cfg4.err; exit 1; }
  unset BLS_BENCH_SHARE_DEVICE
  python3 -c "
import json
for f in ('rehearse_cfg2','rehearse_cfg4'):
  d=json.load(open('$O/'+f+'.json')); print(f, d['n_gpus'], d['value'], d['ms_per_step'], d['data'][-80:])"
fi
if [ -n "$NAPI" ]; then
  # the N-API line: one JS promise per attestation and 1024-set calls, on the adapter's
  # device slots (NAPI_DEVICES, default "0" and "0,0")
  for dv in ${NAPI_DEVICES:-0 0,0}; do
    n=napi_$(echo $dv | tr ',' '_')
    timeout -k 10 400 python -u bench.py --mode napi --devices $dv --steps ${NAPI_STEPS:-8} --warmup 2 > $O/$n.json 2> $O/$n.err || { echo "$n failed"; tail -20 $O/$n.err; exit 1; }
    python3 -c "
import json;d=json.load(open('$O/$n.json'));x=d['napi']
print('$n', d['value'], x['per_set_calls'].get('slot_sets'), x['calls_of_1024_sets']['sets_per_s'])"
  done
fi
if [ -n "$KPROBE" ]; then
  timeout -k 10 120 python -u tools/kprobe.py > $O/kprobe.json 2> $O/kprobe.err || { echo "kprobe failed"; tail -5 $O/kprobe.err; exit 1; }
  cat $O/kprobe.json
fi
if [ -n "$SOLO" ]; then
  # one 32-call pass (32,768 cfg2 sets) alone under a kernel trace (+ SQ counters), per
  # SOLO label "name:VAR=v,..." separated by ";"
  R=$GRAFT_REPO_ROOT
  for ab in $(echo "$SOLO" | tr ';' ' '); do
    label=${ab%%:*}; vars=$(echo "${ab#*:}" | tr ',' ' ')
    PB="python3 $R/bench.py --probe-only --inflight 1 --calls-per-pass ${SOLO_CPP:-32} --steps 1 --warmup 1"
    (cd /tmp && export TMPDIR=/tmp && env $vars timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/$O/solo_$label -o run --output-format csv -- $PB > $R/$O/solo_$label.log 2>&1) || { tail -20 $O/solo_$label.log; exit 1; }
    (cd /tmp && export TMPDIR=/tmp && env $vars timeout -s KILL 120 rocprofv3 --pmc ${SOLO_PMC:-SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE} -d $R/$O/solo_${label}_pmc -o run --output-format csv -- $PB > $R/$O/solo_${label}_pmc.log 2>&1) || { tail -20 $O/solo_${label}_pmc.log; exit 1; }
    python3 -c "
import csv,glob
f=glob.glob('$O/solo_$label/**/*kernel_stats.csv',recursive=True)[0]
for r in csv.DictReader(open(f)):
  n=r['Name'].split('(')[0].replace('void ','')
  if n.startswith(('k_ml','k_chain','k_pre','k_msm','k_gsum')): print('$label', n, r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us')"
  done
fi
if [ -n "$PMC" ]; then
  cd /tmp && export TMPDIR=/tmp
  R=$GRAFT_REPO_ROOT
  P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_LDS"
  P2="SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH"
  P3="GRBM_GUI_ACTIVE GRBM_COUNT"
  P4="FETCH_SIZE"
  P5="WRITE_SIZE"
  PB="python3 $R/bench.py --probe-only --inflight ${PMC_CTX:-16} --calls-per-pass ${PMC_CPP:-22} --steps 1 --warmup 0"
  k=0
  for P in "$P1" "$P2" "$P3" "$P4" "$P5"; do
    k=$((k+1))
    timeout -s KILL 240 rocprofv3 --pmc $P -d $R/$O/pmc$k -o run --output-format csv -- $PB > $R/$O/pmc$k.log 2>&1 || { tail -20 $R/$O/pmc$k.log; exit 1; }
  done
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/$O/trace -o run --output-format csv -- $PB > $R/$O/trace.log 2>&1 || { tail -20 $R/$O/trace.log; exit 1; }
  cd $R
  python3 tools/pmc_summary.py --sets-per-pass $(( ${PMC_CPP:-22} * 1024 )) $O/pmc_summary.json "the timed region's shape: ${PMC_CTX:-16} contexts x ${PMC_CPP:-22} calls of 1024 cfg2 sets, one pass each (bench.py --probe-only --inflight ${PMC_CTX:-16} --calls-per-pass ${PMC_CPP:-22} --steps 1 --warmup 0; the pass shape chosen by the sets in flight as in the timed region); counter collection serialises the kernels, so per-dispatch figures, not the overlap; setup kernels (k_sign, k_sk_to_pk, k_load_pubkeys, k_aggregate) are input synthesis" $O/pmc1 $O/pmc2 $O/pmc3 $O/pmc4 $O/pmc5 > $O/pmc_summary.txt
fi
echo done

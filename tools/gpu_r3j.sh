#!/bin/bash
# round 3: contexts x calls sweep on the one-kernel k_chain build; clean per-kernel SQ / HBM counters and a
# kernel trace of exactly one 32-call pass (--probe-only)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3j
mkdir -p $O
B="python -u bench.py --steps 8 --warmup 1 --no-cpu-baseline --no-sub-records --latency-runs 10"
for cfg in ${CFGS:-"16 8" "12 12" "14 10" "16 10"}; do
  set -- $cfg
  n=r_${1}x${2}
  timeout -k 10 240 $B --inflight $1 --calls-per-pass $2 > $O/$n.json 2> $O/$n.err || { echo "$n failed"; tail -3 $O/$n.err; exit 1; }
  echo "$n $(python3 -c "import json;d=json.load(open('$O/$n.json'));print(d['value'],d['ms_per_step'],d['p50_latency_ms_128'])")"
done
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_LDS"
P2="SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH"
P3="GRBM_GUI_ACTIVE GRBM_COUNT"
P4="FETCH_SIZE"
P5="WRITE_SIZE"
PB="python3 $R/bench.py --probe-only --inflight 1 --calls-per-pass 32 --steps 1 --warmup 0"
k=0
for P in "$P1" "$P2" "$P3" "$P4" "$P5"; do
  k=$((k+1))
  timeout -s KILL 150 rocprofv3 --pmc $P -d $R/$O/pmc$k -o run --output-format csv -- $PB > $R/$O/pmc$k.log 2>&1 || { tail -20 $R/$O/pmc$k.log; exit 1; }
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/$O/trace -o run -- $PB > $R/$O/trace.log 2>&1 || { tail -20 $R/$O/trace.log; exit 1; }
cd $R
python3 tools/pmc_summary.py $O/pmc_summary.json "exactly one pass of 32 cfg2 calls (32768 sets; bench.py --probe-only --inflight 1 --calls-per-pass 32 --steps 1 --warmup 0), split SIMT Miller loops; setup kernels (k_sign, k_sk_to_pk, k_load_pubkeys, k_aggregate) are input synthesis" $O/pmc1 $O/pmc2 $O/pmc3 $O/pmc4 $O/pmc5 > $O/pmc_summary.txt
echo done

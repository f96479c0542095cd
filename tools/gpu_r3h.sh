#!/bin/bash
# round 3: contexts x calls-per-pass sweep for the split SIMT and the cooperative Miller loops,
# then SQ / HBM counter passes over one 32768-set pass (split SIMT default)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3h
mkdir -p $O
B="python -u bench.py --steps 6 --warmup 1 --no-cpu-baseline --no-sub-records --latency-runs 5"
for ml in 0 2; do
  for cfg in ${CFGS:-"2 40" "10 8" "14 8" "16 8"}; do
    set -- $cfg
    n=ml${ml}_${1}x${2}
    BLS_ML_SIMT=$ml timeout -k 10 240 $B --inflight $1 --calls-per-pass $2 > $O/$n.json 2> $O/$n.err || { echo "$n failed"; tail $O/$n.err; exit 1; }
    echo "$n $(python3 -c "import json;d=json.load(open('$O/$n.json'));print(d['value'],d['ms_per_step'])")"
  done
done
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_LDS"
P2="SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH"
P3="GRBM_GUI_ACTIVE GRBM_COUNT"
P4="FETCH_SIZE"
P5="WRITE_SIZE"
# whole-run SIMD utilisation at 14 x 8: VALU-active and wave cycles summed over every kernel
timeout -s KILL 240 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $R/$O/pmc_util -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-sub-records --latency-runs 1 --inflight 14 > $R/$O/pmc_util.log 2>&1 || { echo "pmc util failed"; tail $R/$O/pmc_util.log; exit 1; }
PB="python3 $R/bench.py --no-cpu-baseline --no-sub-records --latency-runs 1 --inflight 1 --calls-per-pass 32 --steps 1 --warmup 1"
k=0
for P in "$P1" "$P2" "$P3" "$P4" "$P5"; do
  k=$((k+1))
  timeout -s KILL 150 rocprofv3 --pmc $P -d $R/$O/pmc$k -o run --output-format csv -- $PB > $R/$O/pmc$k.log 2>&1 || { tail -20 $R/$O/pmc$k.log; exit 1; }
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/$O/trace -o run -- $PB > $R/$O/trace.log 2>&1 || { tail -20 $R/$O/trace.log; exit 1; }
cd $R
python3 tools/pmc_summary.py $O/pmc_summary.json "one pass of 32 cfg2 calls (32768 sets; bench.py --inflight 1 --calls-per-pass 32), split SIMT Miller loops" $O/pmc1 $O/pmc2 $O/pmc3 $O/pmc4 $O/pmc5 > $O/pmc_summary.txt
echo done

#!/bin/bash
# Round-2 baseline on one MI355X: driver-shaped bench, solo kernel trace, and SQ
# counter passes over the cfg2 bench kernel (k_psetn).  Output under gpurun_out/r2b.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r2b
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
B="python3 $R/bench.py --no-cpu-baseline --latency-runs 3"
timeout -k 10 240 $B --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err || { tail -20 $O/bench_driver.err; exit 1; }
cat $O/bench_driver.json
timeout -k 10 240 $B --steps 96 --warmup 2 > $O/bench_96.json 2> $O/bench_96.err || { tail -20 $O/bench_96.err; exit 1; }
cat $O/bench_96.json
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- $B --inflight 1 --steps 6 --warmup 1 > $O/trace.log 2>&1 || { tail -20 $O/trace.log; exit 1; }
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_LDS"
P2="SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH"
P3="GRBM_GUI_ACTIVE GRBM_COUNT"
k=0
for P in "$P1" "$P2" "$P3"; do
  k=$((k+1))
  timeout -s KILL 120 rocprofv3 --pmc $P -d $O/pmc$k -o run --output-format csv -- $B --inflight 1 --steps 4 --warmup 1 > $O/pmc$k.log 2>&1 || { tail -20 $O/pmc$k.log; exit 1; }
done
find $O -name "*.csv" | sort

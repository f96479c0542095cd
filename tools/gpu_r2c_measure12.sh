#!/bin/bash
# Round-2 (third session) measurement set on one MI355X: parity tests, the driver-shaped bench line
# (with the CPU baseline), the N-API mode, a kernel trace with the calls overlapping,
# and SQ / HBM counter passes over one 8192-set call (k_chain: 512 wavefronts,
# k_mlns<8>: 1024 + 128 wavefronts, one signature-sum loop, 6 per CU by LDS).  Everything lands in gpurun_out/meas8.
# $SKIP_TESTS=1 skips the parity tests, $SKIP_BENCH=1 the two bench lines.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/meas8
mkdir -p $O
cd $R
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error" $O/pytest_gpu.log | tail -30; exit 1; }
  tail -1 $O/pytest_gpu.log
fi
if [ -z "$SKIP_BENCH" ]; then
  timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
  cat $O/bench.json
  timeout -k 10 400 python -u bench.py --mode napi --steps 30 --warmup 1 > $O/bench_napi.json 2> $O/bench_napi.err || { echo "napi bench failed"; tail -20 $O/bench_napi.err; }
  cat $O/bench_napi.json
fi
cd /tmp && export TMPDIR=/tmp
B="python3 $R/bench.py --no-cpu-baseline --latency-runs 2"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace16 -o run --output-format csv -- $B --steps 4 --warmup 1 > $O/trace16.log 2>&1 || { tail -20 $O/trace16.log; exit 1; }
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_LDS"
P2="SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH"
P3="GRBM_GUI_ACTIVE GRBM_COUNT"
P4="FETCH_SIZE"
P5="WRITE_SIZE"
k=0
for P in "$P1" "$P2" "$P3" "$P4" "$P5"; do
  k=$((k+1))
  timeout -s KILL 150 rocprofv3 --pmc $P -d $O/pmc$k -o run --output-format csv -- $B --sets 8192 --inflight 1 --calls-per-pass 1 --steps 1 --warmup 1 > $O/pmc$k.log 2>&1 || { tail -20 $O/pmc$k.log; exit 1; }
done
cd $R
python3 tools/pmc_summary.py $O/pmc_summary.json "one 8192-set cfg2 call (bench.py --sets 8192 --inflight 1): k_chain 512 wavefronts (256 VGPRs, 2 per SIMD), k_mlns<8> 1152 wavefronts (1024 shared 8-pair loops + 128 for the signature sums, one of them live: merged signature sum; 166 VGPRs, 6 per CU by LDS)" $O/pmc1 $O/pmc2 $O/pmc3 $O/pmc4 $O/pmc5
python3 tools/trace_timeline.py $(find $O/trace16 -name "*kernel_trace.csv" | head -1) k_mln > $O/timeline.txt
cat $O/timeline.txt

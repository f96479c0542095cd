#!/bin/bash
# k_chain capped at 256 VGPRs (two wavefronts per SIMD, spills) vs the default build.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/occ2
mkdir -p $O; cd $R
V=$R/lodestar_amd/_native/liblodestar_bls_chain_occ2.so
LODESTAR_BLS_LIB=$V BLS_DEBUG_SYNC=1 timeout -k 10 90 python -u tools/sigagg_probe.py 1024 > $O/probe.log 2>&1 || { echo "occ2 probe failed"; tail -20 $O/probe.log; exit 1; }
grep -E "k_chain|valid|invalid" $O/probe.log | head -4
for rep in 1 2; do
  for v in occ2 base; do
    if [ $v = occ2 ]; then export LODESTAR_BLS_LIB=$V; else unset LODESTAR_BLS_LIB; fi
    timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --latency-runs 4 --no-cpu-baseline > $O/bench_${v}_$rep.json 2> $O/bench_${v}_$rep.err || { echo "bench $v failed"; tail -5 $O/bench_${v}_$rep.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/bench_${v}_$rep.json'));print('$v', round(d['value']), d['ms_per_step'], d['p50_latency_ms_128'], d['stage_ms']['per_set'])"
  done
done

#!/bin/bash
# k_chain register budget at the 8 x 8 bench default: 2 waves/SIMD (default build,
# 256 VGPRs with spills), 1 (variant chain_occ1, no cap), 3 (variant chain_occ3).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/chainocc
mkdir -p $O; cd $R
N=$R/lodestar_amd/_native
for rep in 1 2; do
  for v in occ2 occ1 occ3; do
    case $v in
      occ2) L=$N/liblodestar_bls.so;;
      occ1) L=$N/liblodestar_bls_chain_occ1.so;;
      occ3) L=$N/liblodestar_bls_chain_occ3.so;;
    esac
    LODESTAR_BLS_LIB=$L timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --latency-runs 2 --no-cpu-baseline > $O/bench_${v}_$rep.json 2> $O/bench_${v}_$rep.err || { echo "bench $v failed"; tail -5 $O/bench_${v}_$rep.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/bench_${v}_$rep.json'));print('$v', round(d['value']), d['ms_per_step'], d['p50_latency_ms_128'])"
  done
done

#!/bin/bash
# 28-bit-digit Montgomery product (default build) vs the 32-bit-digit one
# (liblodestar_bls_mul32.so, python -m lodestar_amd.build --variant mul32): GPU parity
# on the new build, then the product probe and the cfg2 line of each, interleaved.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/d28
mkdir -p $O; cd $R
BLS_DEBUG_SYNC=1 timeout -k 10 90 python -u tools/sigagg_probe.py 1024 > $O/probe_d28.log 2>&1 || { echo "d28 probe failed"; tail -30 $O/probe_d28.log; exit 1; }
tail -2 $O/probe_d28.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 100 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Timeout|Error|assert" $O/pytest_gpu.log | tail -30; exit 1; }
tail -1 $O/pytest_gpu.log
M32=$R/lodestar_amd/_native/liblodestar_bls_mul32.so
timeout -k 10 200 python -u tools/fpm_probe.py > $O/fpm_d28.json 2>&1 || { cat $O/fpm_d28.json; exit 1; }
LODESTAR_BLS_LIB=$M32 timeout -k 10 200 python -u tools/fpm_probe.py > $O/fpm_mul32.json 2>&1 || { cat $O/fpm_mul32.json; exit 1; }
python3 -c "
import json
for t in ('d28','mul32'):
    d=json.load(open('$O/fpm_'+t+'.json')); print(t, {k:(v if not isinstance(v,dict) else (v['ns_per_fpm_per_lane'], v['Gfpm_per_s'])) for k,v in d.items()})"
for rep in 1 2; do
  for v in d28 mul32; do
    if [ $v = mul32 ]; then export LODESTAR_BLS_LIB=$M32; else unset LODESTAR_BLS_LIB; fi
    timeout -k 10 300 python -u bench.py --steps 16 --warmup 3 --latency-runs 10 --no-cpu-baseline > $O/bench_${v}_$rep.json 2> $O/bench_${v}_$rep.err || { echo "bench $v failed"; tail -5 $O/bench_${v}_$rep.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/bench_${v}_$rep.json'));print('$v', round(d['value']), d['ms_per_step'], d['p50_latency_ms_128'], d['stage_ms'])"
  done
done

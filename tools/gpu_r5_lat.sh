#!/bin/bash
# Round-5 latency A/B on the GPU box: GPU tests on the current build, then the 128-set
# call (p50_latency_ms_128) and the interpreter's per-program step times for the saved
# base build (liblodestar_bls_base.so + coop_tables_base.bin.gz) and the current one.
#   TAG=name (gpurun_out/<TAG>), NOTESTS=1 skips the tests
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r5lat}; mkdir -p $O
N=$GRAFT_REPO_ROOT/lodestar_amd/_native
if [ -z "$NOTESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
  tail -1 $O/pytest.log
fi
for lib in base new; do
  if [ $lib = base ]; then export LODESTAR_BLS_LIB=$N/liblodestar_bls_base.so BLS_COOP_TABLES=$N/coop_tables_base.bin.gz
  else unset LODESTAR_BLS_LIB BLS_COOP_TABLES; fi
  timeout -k 10 180 python -u tools/lat_probe.py --runs 30 > $O/lat_$lib.json 2> $O/lat_$lib.err || { echo "lat $lib failed"; tail -5 $O/lat_$lib.err; exit 1; }
  echo "$lib $(cat $O/lat_$lib.json)"
  timeout -k 10 180 python -u tools/coop_probe.py > $O/coop_$lib.json 2> $O/coop_$lib.err || { echo "coop $lib failed"; tail -5 $O/coop_$lib.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/coop_$lib.json'));print('$lib',{k:v['ms_per_run'] for k,v in d.items() if k.endswith('@1')})"
done

#!/bin/bash
# A/B of the failing-pass Miller loops on the cfg5 slice, alternated, after the GPU tests:
# "off" sets $OFF_VAR=0 (default BLS_MLF_ALONE: the first pass's items per lane, as
# before; BLS_COOP_ML_MAX: the SIMT pair instead of the cooperative loops).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r5fb}; mkdir -p $O
if [ -z "$NOTESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
  tail -1 $O/pytest.log
fi
for ab in off on off2 on2; do
  case $ab in off*) export ${OFF_VAR:-BLS_MLF_ALONE}=${OFF_VAL:-0};; *) unset ${OFF_VAR:-BLS_MLF_ALONE};; esac
  timeout -k 10 300 python -u tools/cfg5_probe.py ${ARGS} > $O/probe_$ab.json 2> $O/probe_$ab.err || { echo "probe $ab failed"; tail -20 $O/probe_$ab.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/probe_$ab.json'));print('$ab',{k:(d[k]['sets_per_s'],d[k]['merged_fail'],d[k]['stage_ms_sum']) for k in ('invalid','valid')})"
done

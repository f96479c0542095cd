#!/bin/bash
# Round-6 failing-pass A/B on the GPU box: tools/sub_probe.py (the cfg4 per-set-request
# slice and the cfg5 slice with invalid sets) per label "name:VAR=v,..." in $ENVS
# (";"-separated), optionally the GPU tests first (TESTS=1) and the N-API bench alone
# (NAPIDBG=1: node benchNapi.js directly, exit status kept).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r6f}; mkdir -p $O
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${TESTK:+-k "$TESTK"} > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
  tail -1 $O/pytest.log
fi
if [ -n "$NAPIDBG" ]; then
  timeout -k 10 300 python -u tools/napi_debug.py > $O/napidbg.json 2> $O/napidbg.err; rc=$?
  echo "napi debug rc=$rc"; tail -c 1500 $O/napidbg.json; tail -20 $O/napidbg.err
fi
for ab in $(echo "${ENVS}" | tr ';' ' '); do
  label=${ab%%:*}; vars=$(echo "${ab#*:}" | tr ',' ' ')
  env $vars timeout -k 10 400 python -u tools/sub_probe.py ${ONLY:+--only $ONLY} > $O/sub_$label.json 2> $O/sub_$label.err || { echo "$label failed"; tail -5 $O/sub_$label.err; exit 1; }
  python3 -c "
import json;d=json.load(open('$O/sub_$label.json'))
print('$label', {k:(v.get('sets_per_s'),v.get('steady_sets_per_s')) for k,v in d.items() if isinstance(v,dict) and 'sets_per_s' in v})"
done
echo done

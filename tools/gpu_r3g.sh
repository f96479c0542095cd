#!/bin/bash
# round 3: probe of the sigagg individual-pass verdict bug, per Miller-loop kernel choice
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3g
mkdir -p $O
for v in 2 1 0; do
  BLS_ML_SIMT=$v timeout -k 10 200 python -u tools/dbg_many.py > $O/simt$v.txt 2>&1 || { echo "probe $v failed"; tail $O/simt$v.txt; exit 1; }
done
echo done

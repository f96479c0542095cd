#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/exp
mkdir -p $O; cd $R
run() { tag=$1; shift; env "$@" timeout -k 10 300 python -u bench.py --steps 12 --warmup 3 --latency-runs 2 --no-cpu-baseline $EXTRA > $O/$tag.json 2> $O/$tag.err || { echo "fail $tag"; tail -5 $O/$tag.err; return 1; }; python3 -c "import json;d=json.load(open('$O/$tag.json'));print('$tag', round(d['value']), d['ms_per_step'])"; }
EXTRA="--inflight 20" run pack4_if20 BLS_ML_PACK=4 && EXTRA="--inflight 20" run pack2_if20 BLS_ML_PACK=2 && EXTRA="--inflight 24" run pset_if24 BLS_SIGAGG=0 && EXTRA="--inflight 16" run pset_if16 BLS_SIGAGG=0 && EXTRA="--inflight 20" run pset_if20 BLS_SIGAGG=0

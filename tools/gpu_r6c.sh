set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6c; mkdir -p $O
R=$GRAFT_REPO_ROOT
timeout -k 10 400 python -u tools/sub_probe.py --detail --only cfg4_slice_batchable,cfg5_slice > $O/detail.json 2> $O/detail.err || { echo "detail failed"; tail -5 $O/detail.err; exit 1; }
cat $O/detail.json
timeout -k 10 400 python -u bench.py --mode napi --steps 8 --warmup 2 > $O/napi_0.json 2> $O/napi_0.err; rc=$?
echo "napi rc=$rc"; tail -c 600 $O/napi_0.json; tail -5 $O/napi_0.err
timeout -k 10 400 python -u bench.py --mode napi --devices 0,0 --steps 8 --warmup 2 > $O/napi_00.json 2> $O/napi_00.err; rc=$?
echo "napi00 rc=$rc"; tail -c 600 $O/napi_00.json; tail -5 $O/napi_00.err
echo done

set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5n; mkdir -p $O
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
python3 -c "
import json;d=json.load(open('$O/bench.json'))
print('bench', d['value'], d['ms_per_step'], d.get('p50_latency_ms_128'), d['roofline']['frac'], d['roofline'].get('frac_fixed'))
print({k:(d[k].get('sets_per_s'),d[k].get('steady_sets_per_s'),d[k].get('p50_ms')) for k in ('cfg3','cfg4_slice','cfg4_slice_batchable','cfg5_slice') if k in d})
print({k:d[k].get('sets_per_s') for k in d if k.startswith('hw_queues')})"
timeout -k 10 400 python -u bench.py --mode napi --steps 8 --warmup 2 > $O/napi.json 2> $O/napi.err || { echo "napi failed"; tail -20 $O/napi.err; exit 1; }
head -c 1500 $O/napi.json

set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6e; mkdir -p $O
timeout -k 10 400 python -u tools/sub_probe.py --detail --only cfg4_slice_batchable,cfg5_slice > $O/detail.json 2> $O/detail.err || { echo "detail failed"; tail -5 $O/detail.err; exit 1; }
cat $O/detail.json; echo
for ab in "gt4:BLS_GROUP_TEST_MIN=4" "gt8:BLS_GROUP_TEST_MIN=8" "base:"; do
  label=${ab%%:*}; vars=$(echo "${ab#*:}" | tr ',' ' ')
  env $vars timeout -k 10 400 python -u tools/sub_probe.py --only cfg4_slice_batchable,cfg5_slice > $O/sub_$label.json 2> $O/sub_$label.err || { echo "$label failed"; tail -5 $O/sub_$label.err; exit 1; }
  python3 -c "
import json;d=json.load(open('$O/sub_$label.json'))
print('$label', {k:(v.get('sets_per_s'),v.get('steady_sets_per_s')) for k,v in d.items() if isinstance(v,dict) and 'sets_per_s' in v})"
done

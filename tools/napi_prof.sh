#!/bin/bash
# The N-API per-attestation leg under Node's CPU profiler (--cpu-prof): where the main
# thread's time goes.  Writes gpurun_out/$TAG/*.cpuprofile and a self-time summary.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r6prof}
mkdir -p $O
timeout -k 10 300 python -u - "$O" <<'PY' || exit 1
import json, sys
sys.path.insert(0, ".")
import bench
from lodestar_amd.native import GpuContext
o = sys.argv[1]
gpu = GpuContext(0)
w = bench.make_workload(gpu, 1024 * 22, 0, 0)
sets = w[2]
pks48 = gpu.sk_to_pk(b"".join(bench.interop_sk(i) for i in range(len(sets)))).tobytes()
gpu.close()
open(o + "/work.json", "w").write(json.dumps({"pubkeys48": pks48.hex(), "sets": [
    {"idx": pk[0], "msg": m.hex(), "sig": s.hex()} for pk, m, s in sets]}))
PY
UV_THREADPOOL_SIZE=18 timeout -k 10 300 node --cpu-prof --cpu-prof-dir=$O integration/js/benchNapi.js $O/work.json 4 16 22528 1 22528 0 > $O/bench.json 2> $O/bench.err || exit 1
rm -f $O/work.json
python3 - "$O" <<'PY'
import glob, json, sys, collections
o = sys.argv[1]
f = sorted(glob.glob(o + "/*.cpuprofile"))[-1]
p = json.load(open(f))
nodes = {n["id"]: n for n in p["nodes"]}
dt = collections.Counter()
for sid, d in zip(p["samples"], p["timeDeltas"]):
    n = nodes[sid]["callFrame"]
    dt[(n["functionName"] or "(anon)", n["url"].split("/")[-1], n["lineNumber"])] += d
tot = sum(dt.values())
out = [{"fn": k[0], "file": k[1], "line": k[2], "self_ms": round(v / 1e3, 1), "pct": round(100 * v / tot, 1)} for k, v in dt.most_common(25)]
json.dump({"total_ms": round(tot / 1e3, 1), "top": out}, open(o + "/summary.json", "w"), indent=1)
print(json.dumps(out[:25], indent=0))
PY

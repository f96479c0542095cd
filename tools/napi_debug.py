"""The N-API bench leg (bench.py --mode napi) with the Node child's exit status kept:
the cfg2 work file as bench.py makes it, then benchNapi.js at growing sizes; prints one
JSON object per run (exit status, signal, the tail of stderr, the line if any)."""
import json
import os
import shutil
import subprocess
import sys
import tempfile
from pathlib import Path

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import bench  # noqa: E402


def main():
    from lodestar_amd.native import GpuContext

    node = shutil.which("node")
    out = {}
    with tempfile.TemporaryDirectory() as td:
        gpu = GpuContext(0)
        w = bench.make_workload(gpu, 1024 * 22, 0, 0)
        sets = w[2]
        pks48 = gpu.sk_to_pk(b"".join(bench.interop_sk(i) for i in range(len(sets)))).tobytes()
        gpu.close()
        wf = Path(td) / "work.json"
        wf.write_text(json.dumps({"pubkeys48": pks48.hex(),
                                  "sets": [{"idx": pk[0], "msg": m.hex(), "sig": s.hex()} for pk, m, s in sets]}))
        ctx = os.environ.get("NAPI_CTX", "16")
        runs = os.environ.get("NAPI_RUNS", "small,batched,per_set").split(",")
        cfgs = {"small": ["2", "2", "4096", "1", "1024", "0"],
                "batched": ["8", ctx, str(len(sets)), "1024", str(len(sets)), "0"],
                "per_set": ["8", ctx, str(len(sets)), "1", str(len(sets)), "0"]}
        for name in runs:
            args = cfgs[name.rstrip("0123456789")]
            # BLS_NAPI_SEGV_TRACE: the addon prints a native backtrace on a fatal signal
            env = dict(os.environ, UV_THREADPOOL_SIZE=str(int(ctx) + 2), BLS_NAPI_SEGV_TRACE="1")
            flags = os.environ.get("NODE_FLAGS", "").split()  # e.g. --max-semi-space-size=64
            p = subprocess.run([node, *flags, str(bench.ROOT / "integration" / "js" / "benchNapi.js"), str(wf), *args],
                               capture_output=True, text=True, env=env, timeout=240)
            out[name] = {"rc": p.returncode, "stderr": p.stderr[-8000:], "stdout": p.stdout[-600:]}
            print(name, p.returncode, file=sys.stderr, flush=True)
            if p.returncode != 0:
                break
    print(json.dumps(out))


if __name__ == "__main__":
    main()

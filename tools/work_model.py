#!/usr/bin/env python3
"""Build and run tools/work_model.cpp (host g++, the product's own bls/*.hpp math with
the Fp-product counter on) and write lodestar_amd/_native/work_model.json, the
algorithmic work per set bench.py prices its roofline with."""
from __future__ import annotations

import json
import subprocess
import sys
import tempfile
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent


def build(out: Path | None = None, verbose: bool = True) -> Path:
    out = out or ROOT / "lodestar_amd" / "_native" / "work_model.json"
    with tempfile.TemporaryDirectory() as td:
        exe = Path(td) / "work_model"
        subprocess.run(["g++", "-O2", "-std=c++17", "-I", str(ROOT / "include"), "-I", str(ROOT / "lodestar_amd" / "csrc"),
                        str(ROOT / "tools" / "work_model.cpp"), "-o", str(exe)], check=True)
        res = json.loads(subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout)
    res["source"] = "tools/work_model.cpp: host-compiled bls/*.hpp, Fp products counted per stage"
    out.parent.mkdir(parents=True, exist_ok=True)
    out.write_text(json.dumps(res, indent=1) + "\n")
    if verbose:
        print("[build] work model ->", out, res, flush=True)
    return out


if __name__ == "__main__":
    build(Path(sys.argv[1]) if len(sys.argv) > 1 else None)

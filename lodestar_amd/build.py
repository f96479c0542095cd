"""In-tree build of the gfx950 HIP library (lodestar_amd/_native/liblodestar_bls.so).

Each kernel lives in its own translation unit (lodestar_amd/csrc/kernels/*.hip) so
the TUs compile in parallel; objects are cached by a hash of the sources, flags
and headers so an unchanged tree relinks in seconds.  Used by
__graft_entry__.build() and runnable directly:  python -m lodestar_amd.build
"""
from __future__ import annotations

import concurrent.futures as cf
import hashlib
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
PKG = ROOT / "lodestar_amd"
CSRC = PKG / "csrc"
OUT_DIR = PKG / "_native"
OBJ_DIR = ROOT / "build" / "obj"
LIB = OUT_DIR / "liblodestar_bls.so"
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"
FLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-I", str(ROOT / "include"), "-I", str(CSRC)]


def _headers_digest() -> str:
    h = hashlib.sha256()
    for p in sorted(list(CSRC.rglob("*.hpp")) + list((ROOT / "include").glob("*.h"))):
        h.update(p.name.encode())
        h.update(p.read_bytes())
    return h.hexdigest()


def sources() -> list[Path]:
    return [CSRC / "bls_gpu.hip"] + sorted((CSRC / "kernels").glob("*.hip"))


# A/B build variants: extra defines -> lodestar_amd/_native/liblodestar_bls_<name>.so
VARIANTS = {"mul32": ["-DBLS_FP_MUL32", "-DBLS_CHAIN_INL32"], "chain_inl32": ["-DBLS_CHAIN_INL32"],
            "chain_occ1": ["-DBLS_CHAIN_OCC1"], "chain_occ3": ["-DBLS_CHAIN_OCC3"],
            "chain_binr": ["-DBLS_CHAIN_BINARY_R"]}


def _compile(src: Path, hdr: str, verbose: bool, extra: list[str] | None = None) -> Path:
    flags = FLAGS + (extra or [])
    key = hashlib.sha256((hdr + " ".join(flags)).encode() + src.read_bytes()).hexdigest()[:16]
    obj = OBJ_DIR / f"{src.stem}.{key}.o"
    if obj.exists():
        return obj
    cmd = [HIPCC, *flags, "-c", str(src), "-o", str(obj) + ".tmp"]
    if verbose:
        print("[build]", " ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(str(obj) + ".tmp", obj)
    return obj


def build_coop_tables(verbose: bool = True) -> Path:
    """Cooperative-kernel program tables (tools/gen_coop.py), regenerated when the
    generator sources change."""
    tools = ROOT / "tools"
    out = OUT_DIR / "coop_tables.bin"
    gz = OUT_DIR / "coop_tables.bin.gz"  # what the library loads and what travels to the GPU box
    key = hashlib.sha256(b"".join((tools / f).read_bytes()
                                  for f in ("gen_coop.py", "gen_pset.py", "circuits.py", "gen_constants.py"))).hexdigest()
    stamp = OUT_DIR / ".coop_stamp"
    if gz.exists() and out.with_name("coop_programs.json").exists() and stamp.exists() and stamp.read_text() == key:
        return gz
    if not (out.exists() and stamp.exists() and stamp.read_text() == key):
        if verbose:
            print("[build] tools/gen_coop.py ->", out, flush=True)
        subprocess.run([sys.executable, str(tools / "gen_coop.py"), str(out)], check=True)
    import gzip

    with open(out, "rb") as src, gzip.open(str(gz) + ".tmp", "wb", compresslevel=6) as dst:
        dst.write(src.read())
    os.replace(str(gz) + ".tmp", gz)
    stamp.write_text(key)
    return gz


def build_work_model(verbose: bool = True) -> Path:
    """Fp products per stage (tools/work_model.py), regenerated when the math changes:
    the algorithmic work bench.py prices its roofline with."""
    out = OUT_DIR / "work_model.json"
    key = hashlib.sha256(_headers_digest().encode() + (ROOT / "tools" / "work_model.cpp").read_bytes()).hexdigest()
    stamp = OUT_DIR / ".work_stamp"
    if out.exists() and stamp.exists() and stamp.read_text() == key:
        return out
    sys.path.insert(0, str(ROOT / "tools"))
    import work_model

    work_model.build(out, verbose)
    stamp.write_text(key)
    return out


def build(jobs: int | None = None, verbose: bool = True, variant: str | None = None) -> Path:
    OUT_DIR.mkdir(parents=True, exist_ok=True)
    OBJ_DIR.mkdir(parents=True, exist_ok=True)
    build_coop_tables(verbose)
    build_work_model(verbose)
    hdr = _headers_digest()
    srcs = sources()
    extra = VARIANTS[variant] if variant else None
    lib = OUT_DIR / f"liblodestar_bls_{variant}.so" if variant else LIB
    jobs = jobs or min(len(srcs), os.cpu_count() or 4)
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        objs = list(ex.map(lambda s: _compile(s, hdr, verbose, extra), srcs))
    stamp = hashlib.sha256("".join(str(o) for o in objs).encode()).hexdigest()
    stamp_file = OUT_DIR / (f".lib_stamp_{variant}" if variant else ".lib_stamp")
    if lib.exists() and stamp_file.exists() and stamp_file.read_text() == stamp:
        return lib
    cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", str(lib) + ".tmp", *map(str, objs), "-lz"]
    if verbose:
        print("[build]", " ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(str(lib) + ".tmp", lib)
    stamp_file.write_text(stamp)
    return lib


def build_hostsim(verbose: bool = True) -> Path:
    """CPU build of the kernels' math for tests/ (test infrastructure, not the product)."""
    src = ROOT / "tests" / "native" / "hostsim.cpp"
    out = ROOT / "tests" / "native" / "libhostsim.so"
    hdr = _headers_digest()
    key = hashlib.sha256(hdr.encode() + src.read_bytes()).hexdigest()[:16]
    stamp = out.with_suffix(".stamp")
    if out.exists() and stamp.exists() and stamp.read_text() == key:
        return out
    cmd = ["g++", "-O2", "-std=c++17", "-shared", "-fPIC", "-DBLS_COUNT_OPS", "-I", str(CSRC), "-I",
           str(ROOT / "include"), "-o", str(out), str(src)]
    if verbose:
        print("[build]", " ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    stamp.write_text(key)
    return out


def build_cpu_baseline(verbose: bool = True) -> Path:
    """The C++ CPU baseline under oracle/cpu (benchmark / test infrastructure, "not
    blst"; oracle/cpu/bls_cpu.cpp), next to its source: bench.py's cpu_baseline leg
    loads it on the GPU box's host cores."""
    out = ROOT / "oracle" / "cpu" / "libbls_cpu.so"
    cmd = ["make", "-s", "-C", str(ROOT / "oracle" / "cpu")]
    if verbose:
        print("[build]", " ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    return out


def build_napi(verbose: bool = True) -> Path | None:
    """N-API addon (integration/napi/lodestar_bls_napi.c) over the C-ABI, next to the
    library; skipped when the Node headers are absent."""
    hdr_dir = Path("/usr/include/node")
    if not (hdr_dir / "node_api.h").exists():
        return None
    src = ROOT / "integration" / "napi" / "lodestar_bls_napi.c"
    out = OUT_DIR / "lodestar_bls.node"
    key = hashlib.sha256(src.read_bytes() + (ROOT / "include" / "lodestar_bls.h").read_bytes()).hexdigest()[:16]
    stamp = OUT_DIR / ".napi_stamp"
    if out.exists() and stamp.exists() and stamp.read_text() == key:
        return out
    cmd = ["gcc", "-O2", "-shared", "-fPIC", "-I", str(hdr_dir), "-I", str(ROOT / "include"), str(src),
           "-L", str(OUT_DIR), "-llodestar_bls", "-Wl,-rpath,$ORIGIN", "-o", str(out)]
    if verbose:
        print("[build]", " ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    stamp.write_text(key)
    return out


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--variant":
        build(variant=sys.argv[2])
        sys.exit(0)
    build(jobs=int(sys.argv[1]) if len(sys.argv) > 1 else None)
    build_napi()
    build_hostsim()
    build_cpu_baseline()

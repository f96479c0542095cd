"""In-tree build of the gfx950 HIP library (lodestar_amd/_native/liblodestar_bls.so).

Each kernel lives in its own translation unit (lodestar_amd/csrc/kernels/*.hip) so
the TUs compile in parallel; objects are cached by a hash of the sources, flags
and headers so an unchanged tree relinks in seconds.  Used by
__graft_entry__.build() and runnable directly:  python -m lodestar_amd.build
"""
from __future__ import annotations

import concurrent.futures as cf
import hashlib
import json
import os
import re
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
# (the round-3 variants that lost were removed from the sources; their A/B records stay
# under profiles/r03_ab_*.json)
VARIANTS: dict[str, list[str] | dict[str, list[str]]] = {
    # (a variant may also give flags per translation unit, {file stem: flags}; LLVM's
    # iterative-ilp / iterative-minreg schedulers on k_mlq.hip alone measured slower /
    # level, profiles/r05_ab_sched_strategy.json)
}


def _variant_flags(variant: str | None, tu: str) -> list[str] | None:
    """extra compiler flags of a build variant for one translation unit (by file stem)"""
    if not variant:
        return None
    v = VARIANTS[variant]
    return v if isinstance(v, list) else v.get(tu) or None


# Scratch: the HIP runtime backs each hardware queue with scratch for a full device of the
# deepest kernel dispatched on it, scratch bytes/lane x 64 x resident waves (occupancy x
# 1024 SIMDs), and past ~8 GiB over the queues in use it aborts them with
# HSA_STATUS_ERROR_OUT_OF_RESOURCES (profiles/r03_scratch_out_of_resources.txt).  The
# library admits contexts at run time against that (bls_gpu_init_priority, the
# per-queue figure baked in as BLS_SCRATCH_PER_QUEUE from the kernels compiled here:
# scratch_per_queue()).  The build refuses a kernel whose reservation alone would leave
# room for fewer than MIN_QUEUES queues within the default 6 GiB admission budget.
ADMISSION_BUDGET = 6 << 30
MIN_QUEUES = 4
SIMDS = 1024


def _resources(remarks: str) -> list[dict]:
    """Per kernel: name, scratch bytes/lane, occupancy (waves/SIMD) from hipcc's
    -Rpass-analysis=kernel-resource-usage remarks."""
    out, cur = [], None
    for line in remarks.splitlines():
        if "remark:" not in line:
            continue
        body = line.split("remark:", 1)[1].strip()
        if body.startswith("Function Name:"):
            cur = {"name": body.split(":", 1)[1].strip().split(" ")[0]}
            out.append(cur)
        elif cur is not None and body.startswith("ScratchSize"):
            cur["scratch"] = int(body.split(":", 1)[1].split()[0])
        elif cur is not None and body.startswith("Occupancy"):
            cur["occupancy"] = int(body.split(":", 1)[1].split()[0])
        elif cur is not None and body.startswith("VGPRs:"):
            cur["vgprs"] = int(body.split(":", 1)[1].split()[0])
        elif cur is not None and body.startswith("AGPRs:"):
            cur["agprs"] = int(body.split(":", 1)[1].split()[0])
    for k in out:
        k["device_scratch_bytes"] = k.get("scratch", 0) * 64 * k.get("occupancy", 1) * SIMDS
    return out


def _check_scratch(src: Path, kernels: list[dict]) -> None:
    cap = ADMISSION_BUDGET // MIN_QUEUES
    for k in kernels:
        if k["device_scratch_bytes"] > cap:
            raise SystemExit(f"{src.name}: kernel {k['name']} reserves {k['device_scratch_bytes'] >> 20} MiB of "
                             f"scratch per queue ({k.get('scratch')} B/lane x 64 x {k.get('occupancy')} waves/SIMD "
                             f"x {SIMDS} SIMDs) > {cap >> 20} MiB: fewer than {MIN_QUEUES} contexts would fit the "
                             "runtime's ~8 GiB (lodestar_amd/build.py ADMISSION_BUDGET)")


# Input-fixture and measurement kernels (signing / key derivation for synthetic inputs,
# the MAD-peak, self-test and latency probes): never launched by a verify call, so they do
# not set the per-queue figure a verifier context is admitted against
FIXTURE_TUS = ("k_sign", "k_probe", "k_peak", "k_selftest")
FIXTURE_KERNELS = ("k_coop_probe",)


def _plain_name(mangled: str) -> str:
    m = re.match(r"_Z(\d+)", mangled)  # the kernel's plain name from its mangled one
    return mangled[m.end(): m.end() + int(m.group(1))] if m else mangled


def scratch_per_queue(table: list[dict]) -> tuple[int, str]:
    """The deepest verify-path kernel's per-queue reservation (bytes) and its name: what a
    context's queue may have to hold (any verify-path kernel can run on a context's
    stream; the fixture and probe kernels, FIXTURE_TUS / FIXTURE_KERNELS, are left out)."""
    path = [k for k in table if k.get("tu") not in FIXTURE_TUS and _plain_name(k["name"]) not in FIXTURE_KERNELS]
    worst = max(path, key=lambda k: k["device_scratch_bytes"])
    # the fixture kernels DO run on verifier contexts' streams (bench and tests sign and
    # probe through them), so admission stays right only while none of them needs more
    # than the verify path's deepest kernel: refuse the build otherwise
    fixtures = [k for k in table if k not in path]
    deepest = max(fixtures, key=lambda k: k["device_scratch_bytes"], default=None)
    if deepest is not None and deepest["device_scratch_bytes"] > worst["device_scratch_bytes"]:
        raise RuntimeError(
            f"fixture kernel {_plain_name(deepest['name'])} reserves {deepest['device_scratch_bytes']} B of scratch per "
            f"queue, more than the verify path's deepest ({_plain_name(worst['name'])}, "
            f"{worst['device_scratch_bytes']} B): the admission figure would under-count; shrink it or count it")
    return worst["device_scratch_bytes"], _plain_name(worst["name"])


def _compile(src: Path, hdr: str, verbose: bool, extra: list[str] | None = None) -> Path:
    flags = FLAGS + (extra or [])
    key = hashlib.sha256((hdr + " ".join(flags)).encode() + src.read_bytes()).hexdigest()[:16]
    obj = OBJ_DIR / f"{src.stem}.{key}.o"
    res = obj.with_suffix(".res.json")
    if obj.exists() and res.exists():
        return obj
    cmd = [HIPCC, *flags, "-Rpass-analysis=kernel-resource-usage", "-c", str(src), "-o", str(obj) + ".tmp"]
    if verbose:
        print("[build]", " ".join(cmd), flush=True)
    p = subprocess.run(cmd, capture_output=True, text=True)
    if p.returncode != 0:
        sys.stderr.write(p.stderr)
        raise subprocess.CalledProcessError(p.returncode, cmd)
    kernels = _resources(p.stderr)
    _check_scratch(src, kernels)
    res.write_text(json.dumps(kernels, indent=1))
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
    lib = OUT_DIR / f"liblodestar_bls_{variant}.so" if variant else LIB
    jobs = jobs or min(len(srcs), os.cpu_count() or 4)
    # the kernels first: their resource usage sets the host TU's admission figure
    kern_srcs, host_src = srcs[1:], srcs[0]
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        kobjs = list(ex.map(lambda s: _compile(s, hdr, verbose, _variant_flags(variant, s.stem)), kern_srcs))
    table = [dict(k, tu=o.stem.split(".")[0]) for o in kobjs for k in json.loads(o.with_suffix(".res.json").read_text())]
    per_queue, worst = scratch_per_queue(table)
    host_extra = (_variant_flags(variant, host_src.stem) or []) + [f"-DBLS_SCRATCH_PER_QUEUE={per_queue}ull",
                                                                  f'-DBLS_SCRATCH_WORST_KERNEL="{worst}"']
    objs = [_compile(host_src, hdr, verbose, host_extra)] + kobjs
    if not variant:  # every kernel's registers, occupancy and scratch reservation, for the record
        (OUT_DIR / "kernel_resources.json").write_text(json.dumps(
            {"scratch_per_queue": per_queue, "scratch_worst_kernel": worst, "kernels": table}, indent=1))
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

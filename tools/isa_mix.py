"""Static instruction mix per function of a gfx950 device assembly file
(hipcc --cuda-device-only -S): total instructions, v_mad_u64_u32, v_accvgpr moves,
scratch loads/stores, calls.  Measurement tool, not part of the product.
usage: python tools/isa_mix.py file.s [name-substring ...]"""
import collections
import re
import sys


def functions(path):
    cur, out = None, {}
    for line in open(path):
        s = line.strip()
        m = re.match(r"^([A-Za-z_.$][\w.$]*):", line)
        if m and not m.group(1).startswith(".L"):
            cur = m.group(1)
            out[cur] = collections.Counter()
            continue
        if cur is None or not s or s.startswith((".", ";", "//")) or s.endswith(":"):
            if s.startswith(".Lfunc_end"):
                cur = None
            continue
        op = s.split()[0]
        out[cur][op] += 1
    return out


def main():
    fs = functions(sys.argv[1])
    pats = sys.argv[2:]
    for name, c in fs.items():
        if pats and not any(p in name for p in pats):
            continue
        tot = sum(c.values())
        if tot == 0:
            continue
        v = sum(n for o, n in c.items() if o.startswith("v_"))
        mad = c["v_mad_u64_u32"] + c["v_mad_i64_i32"]
        acc = sum(n for o, n in c.items() if o.startswith("v_accvgpr"))
        scr = sum(n for o, n in c.items() if o.startswith("scratch_"))
        top = ", ".join(f"{o} {n}" for o, n in c.most_common(12))
        print(f"{name[:60]:60s} tot {tot:6d} valu {v:6d} mad {mad:5d} acc {acc:5d} scratch {scr:4d} call {c['s_swappc_b64']}\n    {top}")


if __name__ == "__main__":
    main()

"""The bench line's committed-evidence fields (bench.py committed_pmc /
committed_kernel_times) and the counter summariser that writes them
(tools/pmc_summary.py): CPU only, no device."""
import csv
import json
import subprocess
import sys
from pathlib import Path

import bench

ROOT = Path(__file__).resolve().parent.parent


def test_committed_pmc_timed_shape_counts_verify_kernels_only():
    p = bench.committed_pmc()
    assert p is not None and p["sets_per_pass"] == 22528
    by = p["valu_wave_insts_per_set_timed_shape_by_kernel"]
    # input-synthesis kernels in the probe (k_sign, k_sk_to_pk, k_load_pubkeys) are not
    # part of a verify pass
    assert all(k.startswith(bench.VERIFY_KERNELS) for k in by)
    assert p["valu_wave_insts_per_set_timed_shape"] == sum(by.values())
    assert 100_000 < p["valu_wave_insts_per_set_timed_shape"] < 200_000
    d = json.loads((ROOT / "profiles" / bench.PMC_FILE).read_text())
    for k, v in by.items():
        assert v == min(d["per_dispatch_valu_wave_insts_per_set"][k])


def test_committed_kernel_times_has_the_roofline_kernels():
    t = bench.committed_kernel_times()
    assert any(k.startswith("k_mlf") for k in t) and "k_chain" in t
    assert all(v > 0 for v in t.values())


def test_pmc_summary_per_dispatch(tmp_path):
    rows = [("void k_chain(bls::PipeBufs)", "SQ_INSTS_VALU", 2 * 1024 * 500),
            ("void k_chain(bls::PipeBufs)", "SQ_INSTS_VALU", 2 * 1024 * 400),
            ("void k_chain(bls::PipeBufs)", "SQ_WAVES", 32),
            ("void k_chain(bls::PipeBufs)", "SQ_WAVES", 32)]
    d = tmp_path / "pmc1"
    d.mkdir()
    with open(d / "run_counter_collection.csv", "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Kernel_Name", "Counter_Name", "Counter_Value"])
        w.writerows(rows)
    out = tmp_path / "s.json"
    subprocess.run([sys.executable, str(ROOT / "tools" / "pmc_summary.py"), "--sets-per-pass", "1024",
                    "--shape", "test shape", str(out), "note", str(d)], check=True, capture_output=True)
    s = json.loads(out.read_text())
    assert s["sets_per_pass"] == 1024 and s["shape"] == "test shape"
    assert s["per_dispatch_valu_wave_insts_per_set"]["k_chain"] == [1000, 800]
    assert s["kernels"]["k_chain"]["SQ_INSTS_VALU"] == 2 * 1024 * 450

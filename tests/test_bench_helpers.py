"""CPU checks of bench.py's bookkeeping helpers (no GPU): the PMC summary
lookup by kernel name or template instance, the tree roofline's handling of
an untimed launch, and the steady-state halves."""
import importlib.util
import json
import math
import os

from conftest import ROOT


def _bench():
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_load_profile_by_template_instance(tmp_path, monkeypatch):
    b = _bench()
    prof = tmp_path / "profiles"
    prof.mkdir()
    (prof / "pmc_summary.json").write_text(json.dumps({
        "k_forest16<2>": {"valu_instr_per_launch": 10.0},
        "k_forest16<4>": {"valu_instr_per_launch": 30.0},
        "k_col_open": {"valu_instr_per_launch": 5.0},
    }))
    monkeypatch.setattr(b, "ROOT", str(tmp_path))
    assert b.load_profile("k_col_open")["valu_instr_per_launch"] == 5.0           # exact key
    assert b.load_profile("k_forest16")["valu_instr_per_launch"] == 30.0          # largest instance
    assert b.load_profile("k_forest16<2>")["valu_instr_per_launch"] == 10.0       # exact instance
    assert b.load_profile("k_layer16") == {}


def test_committed_profile_has_both_tree_kernels():
    b = _bench()
    for k in ("k_layer16", "k_forest16"):
        vi = b.load_profile(k).get("valu_instr_per_launch")
        assert vi and vi > 1e8, k


def test_tree_roofline_untimed_launch_is_null_not_error():
    b = _bench()
    r = b.tree_roofline("k_forest16", 0.0, (1 << 24) - 1)
    assert r["achieved"] is None and r["frac"] is None
    r = b.tree_roofline("k_forest16", 0.6, (1 << 24) - 1)
    assert r["frac"] is not None and 0 < r["frac"] < 1 and 0 < r["frac_mix"] < 1
    assert math.isclose(r["hbm"]["alg_bytes_per_launch"], 72 * ((1 << 24) - 1))


def test_halves():
    b = _bench()
    h = b.halves([1.0, 2.0, 3.0, 4.0], 0.0)
    assert math.isclose(h["first_half"], 1000.0) and math.isclose(h["second_half"], 1000.0)
    assert b.halves([1.0], 0.0) is None

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


def test_stdout_line_is_bounded_and_parseable():
    """the driver could not read round 4's 25.7 KB line. The
    formatter applied to that round's full record must give a json.loads-clean
    line of at most 8 KB that keeps BASELINE's fields, the roofline and the CPU
    baseline (the rest goes to the detail file)."""
    b = _bench()
    full = json.load(open(os.path.join(ROOT, "profiles", "r04", "final", "bench_default.json")))
    assert len(json.dumps(full)) > 20000
    s = json.dumps(b.compact_line(full, "gpurun_out/bench_detail.json"))
    assert len(s) <= b.LINE_MAX_BYTES
    line = json.loads(s)
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "dtype", "config",
              "roofline", "cpu_baseline", "single_proof", "configs", "dist_ntt", "sharded_predicted", "detail"):
        assert k in line, k
    assert line["value"] == full["value"]
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic", "hbm"):
        assert k in line["roofline"], k
    for k in ("value", "cores", "kind", "sample", "gpu_proof_matches_oracle"):
        assert k in line["cpu_baseline"], k
    assert set(line["sharded_predicted"]) == {"2", "4", "8"}


def test_emit_writes_detail_and_bounds_line(tmp_path, capsys):
    b = _bench()
    full = json.load(open(os.path.join(ROOT, "profiles", "r04", "final", "bench_default.json")))
    full["sharded"] = {"value": 1.0, "stages_ms_rank0": {"x" * 40 + str(i): 1.0 for i in range(2000)}}
    det = tmp_path / "d" / "detail.json"
    b.emit(full, str(det))
    printed = capsys.readouterr().out.strip().splitlines()
    assert len(printed) == 1 and len(printed[0]) <= b.LINE_MAX_BYTES
    assert json.loads(printed[0])["detail"] == str(det)
    assert json.load(open(det))["sharded"]["value"] == 1.0

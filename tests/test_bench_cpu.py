"""bench.py's reported figures, checked on the CPU (no GPU run): the SURVEY.md §8d traffic model as
written, the per-stage algorithmic bytes the roofline uses, and the committed closing line of this
round (profiles/<ROUND>_bench.json) against its own inputs -- `value` from the timed steps, the
roofline's achieved rate from the PMC profile it names, the model's fractions from its bytes."""
import json
import os

import pytest

import bench

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_survey_model_as_written():
    # §8d: bytes = P B_G + I B_I + HW B_px with B_G = 312 + 36 M (+ the language feature's 12)
    P, R, HW, M = 1_000_000, 9_000_000, 1920 * 1080, 16
    assert bench.survey_step_bytes(P, R, HW, M, True) == P * (312 + 36 * M + 12) + R * 148 + HW * 64
    # the language step moves fewer per-Gaussian bytes than the full backward
    assert bench.survey_step_bytes(P, R, HW, M, False) < bench.survey_step_bytes(P, R, HW, M, True)


def test_algorithmic_bytes_follow_the_variant():
    P, V, R, HW, M = 1000, 800, 5000, 640 * 360, 16
    full = bench.algorithmic_bytes("render backward", P, V, R, HW, M, color_grad=True, geometry=True)
    lang = bench.algorithmic_bytes("render backward", P, V, R, HW, M, color_grad=False, geometry=False)
    fused = bench.algorithmic_bytes("render backward", P, V, R, HW, M, color_grad=False, geometry=False,
                                    fused_loss=True)
    assert full > lang > fused  # colour gradient and 12-value records; the 1-B code instead of dL/dlang
    assert full - lang == HW * 12 + V * 4 * (12 - 5)
    assert lang - fused == HW * 11
    fwd = bench.algorithmic_bytes("render forward", P, V, R, HW, M)
    assert fwd == R * 52 + HW * 32
    assert bench.algorithmic_bytes("no such stage", P, V, R, HW, M) is None


def _closing():
    path = os.path.join(ROOT, "profiles", f"{bench.ROUND}_bench.json")
    if not os.path.exists(path):
        pytest.skip("no closing bench line of this round committed")
    return json.load(open(path))


def test_closing_line_is_consistent():
    d = _closing()
    assert d["metric"] == bench.METRIC and d["n_gpus"] == 1 and d["higher_is_better"]
    # value = blends per step / seconds per step
    blends = d["config"]["blends_per_step"]
    assert abs(d["value"] - blends / (d["ms_per_step"] * 1e-3)) <= 1e-3 * d["value"]
    # the best of the forms is the one reported
    forms = {k: v for k, v in d["ms_per_step_forms"].items() if v is not None}
    assert d["ms_per_step"] == min(forms.values())
    rf = d["roofline"]
    assert abs(rf["frac"] - rf["achieved"] / rf["peak"]) < 1e-3
    # the VALU rate from the PMC profile the line names and the live launch time it reports
    insts, _, src = bench.pmc_valu(rf["kernel"], "C3")
    assert src == rf["valu_source"] and int(insts) == rf["valu_insts_per_launch"]
    achieved = insts / bench.CUS / (rf["avg_ms"] * 1e-3 * bench.CLOCK_HZ)
    assert abs(achieved - rf["achieved"]) <= 2e-3 * rf["achieved"]
    traffic, tsrc = bench.pmc_traffic(rf["kernel"], "C3")
    # the counter pass may be re-collected after the line was benched: PMC bytes agree to run noise
    assert tsrc == rf["hbm"]["traffic_source"] and abs(traffic - rf["traffic"]) <= 5e-3 * rf["traffic"]
    m = rf["fwd_bwd_model"]
    assert abs(m["frac"] - m["bytes"] / (m["ms"] * 1e-3) / 1e9 / bench.HBM_PEAK_GBS) < 1e-3
    if "step" in m:  # the model bytes over the benched step
        assert m["step"]["ms"] == d["ms_per_step"]
        assert abs(m["step"]["frac"] - m["bytes"] / (d["ms_per_step"] * 1e-3) / 1e9 / bench.HBM_PEAK_GBS) < 1e-3
    cpu = d["cpu_baseline"]
    assert cpu["kind"] in ("port", "reference") and cpu["cores"] >= 1 and cpu["value"] > 0


def test_compulsory_model_and_refused_fractions():
    """the compulsory-bytes model counts a render kernel's record once per visible
    Gaussian and 4 B per instance, never more than the literal §8d bytes once instances outnumber the
    visible Gaussians; a fraction above 1 is refused, naming the model."""
    P, V, R, HW, M = 3_000_000, 2_900_000, 40_000_000, 1920 * 1080, 16
    for stage in ("render forward", "render backward"):
        lit = bench.algorithmic_bytes(stage, P, V, R, HW, M, color_grad=False, geometry=False, fused_loss=True)
        comp = bench.compulsory_bytes(stage, P, V, R, HW, M, color_grad=False, geometry=False, fused_loss=True)
        assert lit - comp == R * 48 - V * 48
    assert bench.compulsory_bytes("preprocess", P, V, R, HW, M) == bench.algorithmic_bytes("preprocess", P, V, R, HW, M)
    assert bench.compulsory_step_bytes(P, V, R, HW, M, False) == \
        bench.survey_step_bytes(P, R, HW, M, False) - 136 * R + 96 * V
    ok = bench.hbm_view(4e9, 1e-3, "m")  # 4 TB/s
    assert ok["frac"] == 0.5 and "frac_refused" not in ok
    bad = bench.hbm_view(9e9, 1e-3, "literal model")
    assert bad["frac"] is None and bad["frac_refused"].startswith("literal model: 1.125")


def _fracs(node, path=""):
    if isinstance(node, dict):
        for k, v in node.items():
            if k == "frac" or k.endswith("_frac"):
                yield f"{path}.{k}", v
            yield from _fracs(v, f"{path}.{k}")


@pytest.mark.parametrize("cfg", ["", "_C5", "_C2"])
def test_committed_lines_have_no_fraction_above_one(cfg):
    """no roofline fraction in this round's committed bench lines exceeds 1 (a
    model whose bytes cannot move in the measured time is refused, and names itself)."""
    path = os.path.join(ROOT, "profiles", f"{bench.ROUND}_bench{cfg}.json")
    if not os.path.exists(path):
        pytest.skip("line not committed")
    d = json.load(open(path))
    for where, f in _fracs(d["roofline"], "roofline"):
        assert f is None or 0.0 < f <= 1.0, (where, f)
    refused = [v for k, v in d["roofline"].items() if isinstance(v, dict) and v.get("frac_refused")]
    for v in refused:
        assert v["frac"] is None and v["model"] in v["frac_refused"]

"""bench.py's roofline fields recomputed from the committed
counter profiles on CPU: the bound is VALU issue, and every fraction the line
reports is a fraction (<= 1) that follows from profiles/pmc_<config>.json --
SQ_INSTS_VALU per launch over the rocprof timed launch average and the wave64
issue ceiling; the algorithmic-byte ratio is reported as a throughput score
beside them.  Where a committed bench line of the same library exists
(profiles/r06_<config>_bench.json, else r05), its fields agree with the profile
within 1 %."""
import glob
import json
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
PROFILES = sorted(glob.glob(os.path.join(REPO, "profiles", "pmc_c*.json")))


def launch_bytes(p, key):
    from vame.metrics import pair_accounting
    w = p["profiled_workload"]
    W, H = (int(x) for x in w["resolution"].split("x"))
    acc = pair_accounting(W, H, (2, 3) if w["modes"] == "2cp+3cp" else (2,))
    pairs = w["pairs_per_step_rank0"]
    return acc[key] * pairs / -(-pairs // 32)


@pytest.mark.parametrize("path", PROFILES, ids=[os.path.basename(p)[:-5] for p in PROFILES])
def test_roofline_fractions_from_profile(path):
    import bench
    p = json.load(open(path))
    pc = p.get("pred_count") or {}
    timed = lambda k: bool((p["kernels"].get(k) or {}).get("timed_avg_ms"))  # noqa: E731
    half, ctu2 = timed("affine_me_half") or timed("affine_me_half2w"), timed("affine_me_ctu2")
    split = timed("affine_me_quad2")  # the quadrant CUs in two kernels (round 6)
    keys = {"affine_me_quad": ("bytes_quad1" if split else "bytes_quad", pc.get("executed_pred_frac_quad")),
            "affine_me_quad2": ("bytes_quad2", pc.get("executed_pred_frac_quad")),
            "affine_me_ctu": (("bytes_half" if ctu2 else "bytes_ctu") if half or ctu2 else "bytes_big",
                              pc.get("executed_pred_frac_ctu")),
            "affine_me_half": ("bytes_half", pc.get("executed_pred_frac_ctu")),
            "affine_me_ctu2": ("bytes_ctu", pc.get("executed_pred_frac_ctu")),
            "affine_me_half2w": ("bytes_half_w", pc.get("executed_pred_frac_ctu")),
            "affine_me_half2": ("bytes_half", pc.get("executed_pred_frac_ctu")),
            "affine_me_half2h": ("bytes_half_h", pc.get("executed_pred_frac_ctu"))}
    seen = 0
    for name, (key, ex) in keys.items():
        k = p["kernels"].get(name) or {}
        t = k.get("timed_avg_ms")
        if not t or "sq_per_launch" not in k:
            continue
        r = bench.kernel_roof(t, launch_bytes(p, key), k, ex)
        insts = k["sq_per_launch"]["SQ_INSTS_VALU"]
        assert r["valu_frac"] == pytest.approx(insts / (t * 1e-3 * 1024 * 2.4e9 * 0.5), rel=1e-12)
        for f in ("valu_frac", "valu_busy", "hbm_measured_frac", "hbm_executed_frac"):
            assert r[f] is not None and 0 < r[f] <= 1, (name, f, r[f])
        assert r["hbm_executed_frac"] == pytest.approx(r["alg_byte_ratio"] * ex, rel=1e-12)
        seen += 1
    assert seen >= 1


@pytest.mark.parametrize("cfg", ["c2", "c3", "c4", "c5"])
def test_committed_line_matches_profile(cfg):
    line_path = os.path.join(REPO, "profiles", f"r06_{cfg}_bench.json")
    if not os.path.exists(line_path):
        line_path = os.path.join(REPO, "profiles", f"r05_{cfg}_bench.json")
    prof_path = os.path.join(REPO, "profiles", f"pmc_{cfg}.json")
    if not (os.path.exists(line_path) and os.path.exists(prof_path)):
        pytest.skip("no line committed for this config")
    d = json.load(open(line_path))
    p = json.load(open(prof_path))
    roof = d["roofline"]
    if not roof.get("profile_same_library") or \
            (d.get("native") or {}).get("sha256") != (p.get("profiled_workload") or {}).get("native_sha256"):
        pytest.skip("the committed line ran another library than the profile")
    assert roof["bound"] == "valu" and roof["frac"] <= 1 and roof["busy"] <= 1
    q = p["kernels"][roof.get("kernel", "affine_me_quad")]
    want = q["sq_per_launch"]["SQ_INSTS_VALU"] / (q["timed_avg_ms"] * 1e-3 * 1024 * 2.4e9 * 0.5)
    assert roof["frac"] == pytest.approx(want, rel=0.01)
    for f in ("hbm_executed_frac", "hbm_measured_frac"):
        assert roof[f] <= 1
    st = roof["step"]
    assert st["valu_frac"] is None or st["valu_frac"] <= 1
    assert st["hbm_executed_frac"] is None or st["hbm_executed_frac"] <= 1

"""Measurement hygiene (CPU): the committed profiles under profiles/ describe the
kernels as they are in this tree, so bench.py's `traffic` / `limiter` fields and
DESIGN.md's per-kernel table are not quoted from code that no longer exists
(measurement item)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


import pytest  # noqa: E402

WORKLOADS = ("C1", "C2", "C2hot", "C3", "C4", "C5")


@pytest.mark.parametrize("w", ["C1", "C2", "C2hot", "C3", "C4", "C5"])
def test_profiles_match_sources(w):
    import bench
    path = os.path.join(ROOT, "profiles", f"{bench.PROFILE_ROUND}_{w}_pmc_summary.json")
    with open(path) as f:
        prof = json.load(f)
    assert prof["source_sha"] == bench.source_sha(), (
        f"{path} was measured on other kernel sources: re-run tools/pmc.sh {bench.PROFILE_ROUND} {w} on the GPU")
    assert prof["chain"]["bytes_per_step"] > 0


def test_c2_profile_covers_every_kernel():
    import bench
    with open(os.path.join(ROOT, "profiles", f"{bench.PROFILE_ROUND}_C2_pmc_summary.json")) as f:
        prof = json.load(f)
    # every chain kernel of the C2 bench has counters and a limiter
    for k in ("eq", "xover", "comp_rms", "comp_describe", "comp_pass0", "comp_fix", "comp_apply", "kweight",
              "finalize"):
        assert prof["kernels"][k]["bytes_per_launch"] > 0 and prof["kernels"][k]["limiter"], k


def test_bench_lines_carry_the_contract_fields():
    import bench
    for w in WORKLOADS:
        with open(os.path.join(ROOT, "profiles", f"{bench.PROFILE_ROUND}_bench_{w}.json")) as f:
            d = json.load(f)
        for key in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
                    "scaling", "vs_baseline", "dtype", "data", "config", "roofline"):
            assert key in d, (w, key)
        r = d["roofline"]
        assert r["unit"] == "GB/s" and r["peak"] == 8000.0
        assert abs(r["frac"] - r["achieved"] / r["peak"]) < 1e-12
        assert abs(d["value"] * d["ms_per_step"] / 1e3 - d["config"]["frames_per_rank_step"] * d["n_gpus"]) \
            <= 1e-6 * d["value"]
        dk = r["dominant_kernel"]  # 16 B per stereo frame over the launch's frames
        frames = d["config"]["frames_per_rank_step"]
        assert abs(dk["algorithmic_bytes_per_launch"] * dk["launches_per_step"] - 16 * frames) <= 1e-6 * 16 * frames
        assert abs(dk["frac"] - dk["algorithmic_bytes_per_launch"] / (dk["avg_launch_ms"] / 1e3) / 1e9 / 8000.0) \
            <= 1e-9
        assert r["traffic"] is not None, w  # every line carries PMC traffic (C1 too since round 5)
        v = r["valu"]  # the VALU floor beside the HBM one
        assert v["lane_instr_per_frame"] > 0 and abs(v["frac"] - v["floor_ms"] / d["ms_per_step"]) < 1e-9, w
    with open(os.path.join(ROOT, "profiles", f"{bench.PROFILE_ROUND}_bench_C2.json")) as f:
        c2 = json.load(f)
    assert c2["roofline"]["traffic"] is not None and c2["cpu_baseline"]["cores"] >= 1

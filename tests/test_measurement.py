"""Measurement hygiene (CPU): the committed profiles under profiles/ describe the
kernels as they are in this tree, so bench.py's `traffic` / `limiter` fields and
DESIGN.md's per-kernel table are not quoted from code that no longer exists
(measurement item)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def test_c2_profile_matches_sources():
    import bench
    with open(os.path.join(ROOT, "profiles", "r03_C2_pmc_summary.json")) as f:
        prof = json.load(f)
    assert prof["source_sha"] == bench.source_sha(), (
        "profiles/r03_C2_pmc_summary.json was measured on other kernel sources: "
        "re-run tools/pmc.sh r03 C2 on the GPU and tools/pmc_summary.py here")
    # every chain kernel of the C2 bench has counters and a limiter
    for k in ("eq", "xover", "comp_rms", "comp_links", "comp_describe", "comp_pass0", "comp_fix", "comp_apply", "kweight",
              "finalize"):
        assert prof["kernels"][k]["bytes_per_launch"] > 0 and prof["kernels"][k]["limiter"], k


def test_bench_lines_carry_the_contract_fields():
    for w in ("C1", "C2", "C2hot", "C3", "C4", "C5"):
        with open(os.path.join(ROOT, "profiles", f"r03_bench_{w}.json")) as f:
            d = json.load(f)
        for key in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
                    "scaling", "vs_baseline", "dtype", "data", "config", "roofline"):
            assert key in d, (w, key)
        r = d["roofline"]
        assert r["unit"] == "GB/s" and r["peak"] == 8000.0
        assert abs(r["frac"] - r["achieved"] / r["peak"]) < 1e-12
        assert abs(d["value"] * d["ms_per_step"] / 1e3 - d["config"]["frames_per_rank_step"] * d["n_gpus"]) \
            <= 1e-6 * d["value"]
    with open(os.path.join(ROOT, "profiles", "r03_bench_C2.json")) as f:
        c2 = json.load(f)
    assert c2["roofline"]["traffic"] is not None and c2["cpu_baseline"]["cores"] >= 1

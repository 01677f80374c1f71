"""DESIGN.md §4's per-kernel floor table from a PMC summary.

Per kernel of the chain: measured us per step (kernel trace), PMC bytes per step,
the HBM floor (those bytes at the 6.3 TB/s a streaming copy reaches on MI355X),
lane-instructions per stereo frame (SQ_INSTS_VALU x 64 x launches / frames), the
VALU floor (those instructions at 39.3 T lane-instr/s: 1024 SIMDs x 16 lanes x 2.4
GHz), the f64 operations the exact arithmetic itself needs per stereo frame (an
analytic count, csrc/ comments), and which floor binds.  Chain totals, and the HBM
fraction the chain could reach if it ran at its VALU floor.

Usage: python tools/floor_table.py profiles/r05_C2_pmc_summary.json <frames per step>
"""
import json
import sys

HBM_COPY = 6.3e12          # B/s, measured streaming copy (MI355X_MICROARCH.md)
LANE_OPS = 1024 * 16 * 2.4e9
ALGO_BYTES_PER_FRAME = 16
# f64 operations per stereo frame the exact recurrences need (two lanes = L, R):
MIN_F64 = {
    "eq": "112 (cascade: 4 x 5 fused pass 1 + 4 x 9 scipy-order pass 2, x2 ch) + width 8",
    "xover": "112 (same for LP2+HP2) + mid 4 + 3 quantise muls x2",
    "kweight": "~22 (mono: 2 x 5 fused + 2 x 9 scipy + energy)",
    "comp_rms": "~39 (3 bands x: rms check 3, window sum 4, release summary 6)",
    "comp_describe": "2 JB = 16 reference walks per active tile frame (active tiles only)",
    "comp_pass0": "~8 per band-frame walked (2 Markstein divisions + step)",
    "comp_fix": "~8 per re-walked band-frame (serial chains)",
    "comp_apply": "~45 (3 bands x: divisions 6, step 3, gain 10^(-att/20) when it moves, 2 x audioop.mul)",
    "finalize": "~10 (gain, soft limiter, quantise x2)",
}


def main():
    prof = json.load(open(sys.argv[1]))
    frames = float(sys.argv[2])
    ks = prof["kernels"]
    rows = []
    tot = {"us": 0.0, "mb": 0.0, "hbm": 0.0, "lane": 0.0, "valu": 0.0}
    for k, q in sorted(ks.items(), key=lambda kv: -(kv[1].get("avg_ns") or 0) * kv[1].get("launches_per_step", 1)):
        lps = q.get("launches_per_step", 1.0)
        us = (q.get("avg_ns") or 0.0) * lps / 1e3
        b = (q.get("bytes_per_launch") or 0.0) * lps
        n = (q.get("sq") or {}).get("SQ_INSTS_VALU") or 0.0
        lane = n * 64 * lps / frames
        hbm_us = b / HBM_COPY * 1e6
        valu_us = lane * frames / LANE_OPS * 1e6
        bind = "VALU" if valu_us >= hbm_us else "HBM"
        rows.append((k, us, b / 1e6, hbm_us, lane, valu_us, MIN_F64.get(k, "—"), bind,
                     us / max(hbm_us, valu_us) if max(hbm_us, valu_us) else float("nan")))
        tot["us"] += us
        tot["mb"] += b / 1e6
        tot["hbm"] += hbm_us
        tot["lane"] += lane
        tot["valu"] += valu_us
    print("| kernel | us / step | PMC MB / step | HBM floor us | lane-instr / stereo frame | VALU floor us "
          "| f64 ops the arithmetic needs / stereo frame | binds | measured / floor |")
    print("|---|---|---|---|---|---|---|---|---|")
    for r in rows:
        print(f"| `{r[0]}` | {r[1]:.1f} | {r[2]:.0f} | {r[3]:.1f} | {r[4]:.0f} | {r[5]:.1f} | {r[6]} | {r[7]} | "
              f"{r[8]:.2f} |")
    print(f"| **chain** | **{tot['us']:.1f}** | **{tot['mb']:.0f}** | {tot['hbm']:.1f} | **{tot['lane']:.0f}** | "
          f"**{tot['valu']:.1f}** | | | {tot['us'] / max(tot['hbm'], tot['valu']):.2f} |")
    algo = ALGO_BYTES_PER_FRAME * frames
    print(f"\nHBM fraction at the chain's VALU floor: {algo / (tot['valu'] * 1e-6) / 8e12:.3f} "
          f"(algorithmic {algo / 1e6:.1f} MB in {tot['valu']:.1f} us); at the measured kernel time: "
          f"{algo / (tot['us'] * 1e-6) / 8e12:.3f}")


if __name__ == "__main__":
    main()

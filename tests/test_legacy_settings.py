"""Settings of the legacy-engine fixtures (mirrors tests/golden/make_golden_legacy.py)."""
LEGACY_FULL = {"saturation": 25.0, "bass_boost": 3.0, "mid_cut": 2.0, "presence_boost": 1.5, "treble_boost": 2.0,
               "width": 1.25, "use_multiband": True, "lufs": -14.0, "low_band_threshold": -20.0,
               "mid_band_threshold": -24.0, "high_band_threshold": -30.0}

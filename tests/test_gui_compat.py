"""GUI engine API (mastering_amd.gui_compat): process_audio / batch_process_audio as
mastering_gui.py:192-232 calls them.  CPU tests swap engine.process for a recorder;
the GPU tests master reference goldens as WAV files through the C-ABI and check
them against the reference's own outputs."""
import os

import numpy as np
import pytest


@pytest.fixture
def fake_engine(monkeypatch):
    from mastering_amd import engine
    calls = []

    def fake_process(src, dst, params, device=0, verbose=False):
        calls.append({"src": src, "dst": dst, "params": dict(params), "device": device})
        if "bad" in os.path.basename(src):
            raise ValueError("Audio must have length greater than the block size.")
        with open(dst, "wb") as f:
            f.write(b"RIFF")
        return {"loudness": -20.0, "gain_db": 6.0, "output_path": dst}

    monkeypatch.setattr(engine, "process", fake_process)
    return calls


GUI_SETTINGS = {  # mastering_gui.py:181-190
    "saturation": 20.0, "bass_boost": 2.0, "mid_cut": 1.0, "presence_boost": 0.5, "treble_boost": 1.5,
    "width": 1.2, "lufs": -14.0, "multiband": True, "compress": False,
    "low_band_threshold": -24.0, "low_band_ratio": 5.0, "mid_band_threshold": -19.0, "mid_band_ratio": 2.5,
    "high_band_threshold": -16.0, "high_band_ratio": 3.5,
}


def test_chain_settings_maps_gui_keys():
    from mastering_amd.gui_compat import chain_settings
    p = chain_settings(dict(GUI_SETTINGS, input_file="a.wav", output_file="b.wav"))
    assert p["low_thresh"] == -24.0 and p["low_ratio"] == 5.0
    assert p["mid_thresh"] == -19.0 and p["mid_ratio"] == 2.5
    assert p["high_thresh"] == -16.0 and p["high_ratio"] == 3.5
    for k in ("input_file", "output_file", "compress", "low_band_threshold"):
        assert k not in p
    assert p["saturation"] == 20.0 and p["lufs"] == -14.0 and p["multiband"] is True


def test_process_audio_statuses(tmp_path, fake_engine):
    from mastering_amd.gui_compat import process_audio
    msgs = []
    s = dict(GUI_SETTINGS, input_file=str(tmp_path / "song.wav"), output_file=str(tmp_path / "out.wav"))
    info = process_audio(s, msgs.append)
    assert info["gain_db"] == 6.0
    assert "complete" in msgs[-1].lower()  # re-enables the GUI's buttons (mastering_gui.py:226)
    assert fake_engine[0]["params"]["low_thresh"] == -24.0
    msgs.clear()
    assert process_audio(dict(s, input_file=str(tmp_path / "bad.wav")), msgs.append) is None
    assert "error" in msgs[-1].lower()
    msgs.clear()
    assert process_audio({"saturation": 0}, msgs.append) is None
    assert "error" in msgs[-1].lower()


def test_batch_empty_folder(tmp_path, fake_engine):
    from mastering_amd.gui_compat import batch_process_audio
    msgs = []
    (tmp_path / "notes.txt").write_text("x")
    assert batch_process_audio(GUI_SETTINGS, str(tmp_path), str(tmp_path / "out"), msgs.append) == {}
    assert "no audio files" in msgs[-1].lower()
    assert not fake_engine


def test_batch_shards_files_over_devices(tmp_path, fake_engine):
    from mastering_amd.gui_compat import batch_process_audio, output_name
    names = [f"t{i:02d}.wav" for i in range(7)] + ["bad.WAV"]
    for n in names:
        (tmp_path / n).write_bytes(b"")
    msgs = []
    res = batch_process_audio(GUI_SETTINGS, str(tmp_path), str(tmp_path / "out"), msgs.append, devices=[0, 1, 2])
    assert sorted(res) == sorted(names)
    assert isinstance(res["bad.WAV"], str) and "ValueError" in res["bad.WAV"]
    assert all(isinstance(res[n], dict) for n in names if n != "bad.WAV")
    by_dev = {}
    for c in fake_engine:
        by_dev.setdefault(c["device"], []).append(os.path.basename(c["src"]))
        assert os.path.basename(c["dst"]) == output_name(c["src"])
    files = sorted(names)  # round-robin over the sorted list (distributed.shard_files)
    for d in (0, 1, 2):
        assert sorted(by_dev[d]) == sorted(files[d::3])
    assert "complete" in msgs[-1].lower() and "error" in msgs[-1].lower()
    assert sum(m.startswith("Processed") for m in msgs) == len(names)


P_HOT_GUI = {  # tests/golden P_HOT in the GUI's keys (mastering_gui.py:181-190)
    "bass_boost": 4.0, "mid_cut": 3.0, "presence_boost": 1.0, "treble_boost": 3.0, "saturation": 30, "width": 1.3,
    "multiband": True, "lufs": -14.0, "compress": False, "low_band_threshold": -16.0, "mid_band_threshold": -21.0,
    "high_band_threshold": -27.0,
}


@pytest.mark.gpu
def test_batch_on_gpu_matches_reference_goldens(tmp_path):
    """batch_process_audio over reference goldens that share one settings dict (P_HOT
    via the GUI's band keys): every output file holds the reference's own output."""
    import json

    from conftest import GOLDEN
    from mastering_amd import gui_compat, wavio
    from test_wav_path import check_against_golden
    src = tmp_path / "in"
    src.mkdir()
    golden = {}
    for name in ("hot_4s", "mono_hot_2s", "hot_96k_1s"):
        d = np.load(os.path.join(GOLDEN, name + ".npz"))
        assert json.loads(str(d["settings"])) == gui_compat.chain_settings({k: v for k, v in P_HOT_GUI.items()})
        wavio.write_wav(str(src / f"{name}.wav"), d["pcm"], int(d["rate"]))
        golden[f"{name}.wav"] = d
    msgs = []
    res = gui_compat.batch_process_audio(P_HOT_GUI, str(src), str(tmp_path / "out"), msgs.append)
    assert "complete" in msgs[-1].lower() and "error" not in msgs[-1].lower()
    for name, d in golden.items():
        got, rate = wavio.read_wav(str(tmp_path / "out" / gui_compat.output_name(name)))
        assert rate == int(d["rate"])
        check_against_golden(got, res[name], d["out"], float(d["loudness"]))


@pytest.mark.gpu
def test_process_audio_on_gpu_matches_reference_golden(tmp_path):
    from conftest import GOLDEN
    from mastering_amd import gui_compat, wavio
    from test_wav_path import check_against_golden
    d = np.load(os.path.join(GOLDEN, "full_4s.npz"))
    wavio.write_wav(str(tmp_path / "a.wav"), d["pcm"], int(d["rate"]))
    s = {"bass_boost": 4.0, "mid_cut": 3.0, "presence_boost": 1.0, "treble_boost": 3.0, "saturation": 30,
         "width": 1.3, "multiband": True, "lufs": -14.0, "input_file": str(tmp_path / "a.wav"),
         "output_file": str(tmp_path / "b.wav")}
    msgs = []
    info = gui_compat.process_audio(s, msgs.append)
    assert "complete" in msgs[-1].lower()
    got, _ = wavio.read_wav(str(tmp_path / "b.wav"))
    check_against_golden(got, info, d["out"], float(d["loudness"]))

"""Worker adapter (mastering_amd.worker): the Pub/Sub push handler of
worker/main.py:15-50 and the object-store flow of AME:24-113 on a local tree.
CPU tests swap engine.process for a recorder; the GPU test masters reference
goldens as objects and checks them against the reference's own outputs."""
import base64
import io
import json
import os

import numpy as np
import pytest


def _envelope(job):
    return {"message": {"data": base64.b64encode(json.dumps(job).encode()).decode()}}


@pytest.fixture
def fake_engine(monkeypatch):
    from mastering_amd import engine
    calls = []

    def fake_process(src, dst, params, device=0, verbose=False):
        calls.append({"src": src, "dst": dst, "params": dict(params)})
        if not os.path.exists(src) or "bad" in os.path.basename(src):
            raise ValueError("Audio must have length greater than the block size.")
        with open(dst, "wb") as f:
            f.write(b"RIFF")
        return {"loudness": -20.0, "gain_db": 6.0}

    monkeypatch.setattr(engine, "process", fake_process)
    return calls


def test_object_path(tmp_path):
    from mastering_amd.worker import object_path
    p, bdir, blob = object_path("gs://bkt/uploads/a.wav", str(tmp_path))
    assert p == str(tmp_path / "bkt" / "uploads" / "a.wav") and bdir == str(tmp_path / "bkt")
    assert blob == "uploads/a.wav"
    for bad in ("gs://bkt", "gs://bkt/", "gs:///x.wav", "gs://bkt/../other/x.wav", "gs://../x.wav",
                "gs://./x.wav", "gs://bkt/./", "gs://bkt/sub/../../x.wav"):
        with pytest.raises(ValueError):
            object_path(bad, str(tmp_path))


def test_push_codes_and_outputs(tmp_path, fake_engine):
    from mastering_amd.worker import handle_push
    root = str(tmp_path)
    (tmp_path / "bkt" / "up").mkdir(parents=True)
    (tmp_path / "bkt" / "up" / "song.wav").write_bytes(b"")
    settings = {"saturation": 10, "multiband": True}
    # malformed envelopes / missing fields -> 400, engine untouched (main.py:21-37)
    assert handle_push(None, root)[1] == 400
    assert handle_push({"nomessage": 1}, root)[1] == 400
    assert handle_push(_envelope({"settings": settings}), root)[1] == 400
    assert handle_push(_envelope({"gcs_uri": "gs://bkt/up/song.wav"}), root)[1] == 400
    assert not fake_engine
    # success -> 204, result + marker under processed/ (AME:92-107)
    assert handle_push(_envelope({"gcs_uri": "gs://bkt/up/song.wav", "settings": settings}), root) == ("", 204)
    out = tmp_path / "bkt" / "processed" / "mastered_song.wav"
    assert out.read_bytes() == b"RIFF"
    assert (tmp_path / "bkt" / "processed" / "mastered_song.wav.complete").read_bytes() == b""
    assert fake_engine[-1]["params"] == settings
    # a failing job is acknowledged (204) and leaves no output or marker (main.py:44-48)
    assert handle_push(_envelope({"gcs_uri": "gs://bkt/up/bad.wav", "settings": settings}), root) == ("", 204)
    assert not (tmp_path / "bkt" / "processed" / "mastered_bad.wav").exists()
    assert not (tmp_path / "bkt" / "processed" / "mastered_bad.wav.complete").exists()
    assert not list((tmp_path / "bkt" / "processed").glob("*.part"))
    # undecodable payload -> acknowledged like any other failure
    assert handle_push({"message": {"data": "!!notbase64"}}, root)[1] == 204


def test_process_raises_like_reference(tmp_path, fake_engine):
    from mastering_amd.worker import process_audio_from_gcs
    with pytest.raises(ValueError):
        process_audio_from_gcs("gs://bkt/missing.wav", {"lufs": -14}, root=str(tmp_path))


def test_wsgi_app(tmp_path, fake_engine, monkeypatch):
    from wsgiref.util import setup_testing_defaults

    from mastering_amd.worker import wsgi_app
    monkeypatch.setenv("MM_BUCKET_ROOT", str(tmp_path))
    (tmp_path / "b").mkdir()
    (tmp_path / "b" / "x.wav").write_bytes(b"")

    def call(method, body):
        env = {}
        setup_testing_defaults(env)
        env.update(REQUEST_METHOD=method, PATH_INFO="/", CONTENT_LENGTH=str(len(body)),
                   **{"wsgi.input": io.BytesIO(body)})
        got = {}
        data = b"".join(wsgi_app(env, lambda s, h: got.update(status=s)))
        return int(got["status"].split()[0]), data

    assert call("POST", json.dumps(_envelope({"gcs_uri": "gs://b/x.wav", "settings": {"lufs": -14}})).encode()) == (204, b"")
    assert (tmp_path / "b" / "processed" / "mastered_x.wav.complete").exists()
    assert call("POST", b"{not json")[0] == 400
    assert call("GET", b"")[0] == 405


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["full_4s", "hot_4s", "nolufs_dubstep_3s"])
def test_worker_job_on_gpu(tmp_path, name):
    """A push job on a reference golden: the object written under processed/ holds the
    reference's own output (AME:24-113 end to end, worker/main.py:15-50)."""
    import json as _json

    from conftest import GOLDEN
    from mastering_amd import wavio
    from mastering_amd.worker import handle_push
    from test_wav_path import check_against_golden
    d = np.load(os.path.join(GOLDEN, name + ".npz"))
    settings = _json.loads(str(d["settings"]))
    (tmp_path / "bkt" / "uploads").mkdir(parents=True)
    wavio.write_wav(str(tmp_path / "bkt" / "uploads" / "track.wav"), d["pcm"], int(d["rate"]))
    env = _envelope({"gcs_uri": "gs://bkt/uploads/track.wav", "settings": settings})
    assert handle_push(env, str(tmp_path)) == ("", 204)
    got, rate = wavio.read_wav(str(tmp_path / "bkt" / "processed" / "mastered_track.wav"))
    assert rate == int(d["rate"])
    from mastering_amd import process
    info = process(str(tmp_path / "bkt" / "uploads" / "track.wav"), str(tmp_path / "again.wav"), settings)
    check_against_golden(got, info, d["out"], float(d["loudness"]))
    assert (tmp_path / "bkt" / "processed" / "mastered_track.wav.complete").exists()

"""Job-queue worker adapter: the reference's Pub/Sub push
handler (worker/main.py:15-50) and its GCS entry point (AME:24-113), with the
object store replaced by a local directory tree.

An object ``gs://<bucket>/<blob>`` lives at ``<root>/<bucket>/<blob>``; ``root``
defaults to ``$MM_BUCKET_ROOT``.  Exactly like AME:92-107, the result is written to
``<bucket>/processed/mastered_<basename(blob)>`` (16-bit WAV) followed by an empty
``.complete`` marker next to it; the marker appears only after the WAV is fully
written (renamed into place), so a poller never sees a partial file.

``wsgi_app`` is the handler as a plain WSGI callable (what gunicorn serves the
reference's Flask app as), so no web framework is needed; ``handle_push`` is the
same logic on a parsed envelope.  Response codes follow worker/main.py: 400 for a
malformed envelope or missing fields, 204 for success AND for a failed job (the
reference acknowledges failures so Pub/Sub does not redeliver them).
"""
from __future__ import annotations

import base64
import json
import os

from . import engine

__all__ = ["object_path", "process_audio_from_gcs", "handle_push", "wsgi_app"]


def object_path(uri: str, root: str | None = None) -> tuple[str, str, str]:
    """``gs://bucket/blob`` -> (local path, bucket dir, blob name), AME:33."""
    root = root if root is not None else os.environ.get("MM_BUCKET_ROOT", ".")
    rest = uri[len("gs://"):] if uri.startswith("gs://") else uri
    if "/" not in rest:
        raise ValueError(f"not an object URI (gs://<bucket>/<blob>): {uri!r}")
    bucket, blob = rest.split("/", 1)
    if not bucket or not blob or blob.endswith("/"):
        raise ValueError(f"not an object URI (gs://<bucket>/<blob>): {uri!r}")
    # a bucket is one path component below the root: no '.', '..' or separators
    if bucket in (".", "..") or os.sep in bucket or (os.altsep and os.altsep in bucket):
        raise ValueError(f"bad bucket name in {uri!r}")
    root_abs = os.path.abspath(root)
    bucket_dir = os.path.join(root, bucket)
    bucket_abs = os.path.abspath(bucket_dir)
    path = os.path.normpath(os.path.join(bucket_dir, blob))
    path_abs = os.path.abspath(path)
    if os.path.commonpath([bucket_abs, root_abs]) != root_abs or bucket_abs == root_abs:
        raise ValueError(f"bucket escapes the object root: {uri!r}")
    if os.path.commonpath([path_abs, bucket_abs]) != bucket_abs or path_abs == bucket_abs:
        raise ValueError(f"object name escapes its bucket: {uri!r}")
    return path, bucket_dir, blob


def process_audio_from_gcs(gcs_uri: str, settings: dict, root: str | None = None, device: int = 0) -> dict:
    """AME:24-113 on the local object tree: master the object, write
    ``processed/mastered_<basename>`` and its ``.complete`` marker; re-raise any
    error after printing it, as the reference does."""
    try:
        src, bucket_dir, blob = object_path(gcs_uri, root)
        print(f"Downloading file from {gcs_uri}...")
        out_name = f"processed/mastered_{os.path.basename(blob)}"
        dst = os.path.join(bucket_dir, out_name)
        os.makedirs(os.path.dirname(dst), exist_ok=True)
        tmp = dst + ".part"
        print("Processing audio in chunks...")
        try:
            info = engine.process(src, tmp, settings, device=device)
            os.replace(tmp, dst)
        finally:
            if os.path.exists(tmp):
                os.remove(tmp)
        print(f"Exporting and uploading processed audio to {out_name}...")
        with open(dst + ".complete", "wb"):
            pass
        print(f"Completion flag created at {out_name}.complete")
        info["output_path"] = os.path.abspath(dst)
        return info
    except Exception as e:
        print(f"FATAL ERROR in mastering engine: {e}")
        raise


def handle_push(envelope, root: str | None = None, device: int = 0) -> tuple[str, int]:
    """worker/main.py:15-50 on a parsed JSON body -> (response body, status)."""
    if not envelope or not isinstance(envelope, dict) or "message" not in envelope:
        print("ERROR: Invalid Pub/Sub message format")
        return "Bad Request: invalid Pub/Sub message format", 400
    try:
        job = json.loads(base64.b64decode(envelope["message"]["data"]).decode("utf-8"))
        gcs_uri = job.get("gcs_uri")
        settings = job.get("settings")
        if not gcs_uri or not settings:
            print(f"ERROR: Missing GCS URI or settings in job data: {job}")
            return "Bad Request: missing GCS URI or settings", 400
        print(f"Starting processing job for {gcs_uri} with settings: {settings}")
        process_audio_from_gcs(gcs_uri, settings, root=root, device=device)
        print(f"Successfully completed processing for {gcs_uri}")
        return "", 204
    except Exception as e:  # acknowledged so the queue does not redeliver (main.py:44-48)
        print(f"CRITICAL ERROR processing job: {e}")
        return "", 204


_REASONS = {204: "204 No Content", 400: "400 BAD REQUEST", 405: "405 METHOD NOT ALLOWED"}


def wsgi_app(environ, start_response):
    """POST / with a Pub/Sub push envelope (JSON) -> handle_push."""
    if environ.get("REQUEST_METHOD") != "POST" or environ.get("PATH_INFO", "/") not in ("", "/"):
        body, status = "Method Not Allowed", 405
    else:
        try:
            n = int(environ.get("CONTENT_LENGTH") or 0)
            envelope = json.loads(environ["wsgi.input"].read(n) or b"null")
        except (ValueError, UnicodeDecodeError):
            envelope = None
        body, status = handle_push(envelope, device=int(os.environ.get("MM_DEVICE", "0")))
    data = body.encode()
    start_response(_REASONS[status], [("Content-Type", "text/html; charset=utf-8"),
                                      ("Content-Length", str(len(data)))])
    return [data]


if __name__ == "__main__":  # python -m mastering_amd.worker  (PORT as in worker/main.py:53)
    from wsgiref.simple_server import make_server
    make_server("0.0.0.0", int(os.environ.get("PORT", 8080)), wsgi_app).serve_forever()

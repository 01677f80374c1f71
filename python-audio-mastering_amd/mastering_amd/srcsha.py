"""Source hash of the HIP library: sha256 over the files the Makefile compiles
(csrc/*.hip, csrc/*.h and include/mastering.h), first 16 hex digits.  The Makefile embeds it in
libmastering_amd.so (mm_source_sha), and smoke() / tests/test_abi.py compare the
loaded library's value with this function's, so a run on the GPU box shows which
sources its library was built from.  Standalone (stdlib only): the Makefile runs
this file as a script."""
import glob
import hashlib
import os

_PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))  # python-audio-mastering_amd/


def library_sha() -> str:
    h = hashlib.sha256()
    # the Makefile's SRC: csrc/*.hip csrc/*.h (a stray file in csrc/ changes neither)
    files = sorted(glob.glob(os.path.join(_PKG, "csrc", "*.hip")) + glob.glob(os.path.join(_PKG, "csrc", "*.h")))
    files.append(os.path.join(os.path.dirname(_PKG), "include", "mastering.h"))
    for f in files:
        h.update(os.path.basename(f).encode())
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


if __name__ == "__main__":
    print(library_sha())

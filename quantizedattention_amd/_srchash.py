"""Content hash of the sources and compile flags libqattn.so is built from.

build.py bakes it into the library (``qattn_source_hash()``, generated ``_build/qattn_version.cpp``)
and rebuilds every object when it changes, whatever the file times say; ``_lib.load()`` compares the
loaded library's hash with the tree's and refuses a stale build.  So a library that travels prebuilt
to another machine runs only if it was linked from exactly the sources beside it.
"""
from __future__ import annotations

import hashlib
from pathlib import Path

_PKG = Path(__file__).resolve().parent
CSRC = _PKG / "csrc"
HEADER = _PKG.parent / "include" / "qattn.h"


def sources() -> list[Path]:
    return sorted(list(CSRC.glob("*.hip")) + list(CSRC.glob("*.h"))) + [HEADER]


def available() -> bool:
    """Whether the sources are present (an installed copy without csrc/ skips the check)."""
    return CSRC.is_dir() and HEADER.exists()


def library_hash() -> str:
    from . import build   # stdlib-only at import: the compile flags
    h = hashlib.sha256()
    for f in sources():
        h.update(f.name.encode())
        h.update(f.read_bytes())
    # the flags, without the machine-specific include path
    flags = [f for f in build.CFLAGS if not f.startswith("-I")]
    h.update(repr((flags, sorted(build.FILE_FLAGS.items()))).encode())
    return h.hexdigest()

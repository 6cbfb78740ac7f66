"""sha256 over the native sources of libmjx355.so: every `.hip` / `.h` file of `csrc/` plus
`include/mjx355.h`, in name order. Standalone (no package imports): the csrc Makefile runs this file
to stamp the hash into the library (`-DMJL_SRC_HASH`, returned by `mjl_version()`), and `_lib.lib()`
refuses a library whose stamp differs from the tree's sources (a stale build).

    python3 _srchash.py          # prints the 16-hex-digit hash of this tree
"""
from __future__ import annotations

import hashlib
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(os.path.dirname(_HERE), "csrc")
HEADER = os.path.join(os.path.dirname(os.path.dirname(_HERE)), "include", "mjx355.h")


def source_hash(csrc: str = CSRC, header: str = HEADER) -> str:
    h = hashlib.sha256()
    files = [os.path.join(csrc, p) for p in sorted(os.listdir(csrc)) if p.endswith((".hip", ".h"))]
    for fp in files + [header]:
        with open(fp, "rb") as f:
            h.update(os.path.basename(fp).encode() + b"\0" + f.read())
    return h.hexdigest()[:16]


if __name__ == "__main__":
    print(source_hash())

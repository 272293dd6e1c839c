"""Which kernel sources a measurement belongs to.

PMC figures (HBM traffic, VALU busy, shading bandwidth) come from separate rocprofv3 passes and
are committed under profiles/; bench.py reports them beside its live numbers only when they were
measured on the kernel sources it is running.  The GPU box gets a snapshot without .git, so the
tag is a content hash of the sources that decide the kernels' code and launch shapes.
"""
from __future__ import annotations

import hashlib
from pathlib import Path

CSRC = Path(__file__).resolve().parent / "csrc"


def kernel_sources_sha(csrc: Path = CSRC) -> str:
    """sha256 (first 16 hex digits) over the HIP sources, their headers and the launch code."""
    h = hashlib.sha256()
    files = sorted(p for p in csrc.iterdir() if p.suffix in (".hip", ".h") or p.name == "pt_capi.cpp")
    for p in files:
        h.update(p.name.encode())
        h.update(b"\0")
        h.update(p.read_bytes())
        h.update(b"\0")
    return h.hexdigest()[:16]

"""PMC provenance: bench.py reports committed PMC figures (HBM traffic,
VALU, shading bandwidth from separate rocprofv3 passes under profiles/) as this tree's only when
they carry the hash of the kernel sources it runs; anything else goes under roofline.pmc_stale."""
from __future__ import annotations

import json
import re
import shutil
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

from optixpathtracer_amd.provenance import CSRC, kernel_sources_sha  # noqa: E402


def _bench():
    import importlib.util

    spec = importlib.util.spec_from_file_location("bench_mod", ROOT / "bench.py")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_sources_sha_tracks_kernel_sources(tmp_path):
    copy = tmp_path / "csrc"
    shutil.copytree(CSRC, copy, ignore=shutil.ignore_patterns("*.o", "*.so"))
    a = kernel_sources_sha(copy)
    assert re.fullmatch(r"[0-9a-f]{16}", a)
    assert a == kernel_sources_sha(CSRC)
    # a kernel edit (one byte in a header) changes the tag; a non-kernel file does not
    (copy / "notes.txt").write_text("not a kernel source")
    assert kernel_sources_sha(copy) == a
    h = copy / "pt_device.h"
    h.write_bytes(h.read_bytes() + b"\n")
    assert kernel_sources_sha(copy) != a


def test_pmc_record_only_current_sources(tmp_path):
    bench = _bench()
    p = tmp_path / "traffic.json"
    assert bench.pmc_record(p, "0123456789abcdef") == (None, False)  # missing
    p.write_text("{not json")
    assert bench.pmc_record(p, "0123456789abcdef") == (None, False)  # unreadable
    p.write_text(json.dumps({"kernel": "k", "sources_sha": "0123456789abcdef"}))
    d, cur = bench.pmc_record(p, "0123456789abcdef")
    assert cur and d["kernel"] == "k"
    d, cur = bench.pmc_record(p, "fedcba9876543210")
    assert not cur and d["sources_sha"] == "0123456789abcdef"
    p.write_text(json.dumps({"kernel": "k"}))  # untagged figures are never current
    assert bench.pmc_record(p, "0123456789abcdef")[1] is False


def test_committed_pmc_files_are_tagged():
    for name in ("traffic.json", "valu.json", "shade_pmc.json", "vmem.json"):
        d = json.loads((ROOT / "profiles" / name).read_text())
        assert re.fullmatch(r"[0-9a-f]{16}", d.get("sources_sha") or ""), name
    v = json.loads((ROOT / "profiles" / "valu.json").read_text())
    # valu_busy counts two wave64 VALU issues per SIMD quad-cycle (pmc_summary.py)
    assert abs(v["valu_busy"] - v["valu_issue_slots"] / 2) < 1e-3
    m = json.loads((ROOT / "profiles" / "vmem.json").read_text())
    assert 0.0 < m["ta_busy"] <= 1.0 and 0.0 < m["td_busy"] <= 1.0

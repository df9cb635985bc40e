"""The tuned GEMM table (sdmi/tuned_gemm.json) the product path reads: well-formed entries, part of the evidence
digest, and an explicit SDMI_TUNED_GEMM that is missing fails instead of silently becoming the split heuristic."""
import json
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "stablediffusion-pytorch_amd")
TABLE = os.path.join(PKG, "sdmi", "tuned_gemm.json")
KEY = re.compile(r"^a[0-2]b[0-2] m\d+ n\d+ k\d+ g\d+x\d+s\d+ i\d+c\d+ x[01]p\d+$")


def test_table_entries_are_well_formed():
    table = json.load(open(TABLE))
    assert table
    for key, e in table.items():
        assert KEY.match(key), key
        splits, variant = (e[0], e[1]) if isinstance(e, list) else (e, 0)
        assert isinstance(splits, int) and 1 <= splits <= 128, (key, e)
        assert isinstance(variant, int) and 0 <= variant <= 11, (key, e)
        k = int(re.search(r" k(\d+) ", key).group(1))
        assert splits <= max(1, (k + 63) // 64), (key, e)  # never more slices than 64-deep k-tiles


def test_table_is_part_of_the_evidence_digest(tmp_path, monkeypatch):
    sys.path.insert(0, PKG)
    from sdmi import _build
    d0 = _build.source_digest()
    t = json.load(open(TABLE))
    k = next(iter(t))
    t[k] = [1, 2] if t[k] != [1, 2] else [2, 2]
    (tmp_path / "tuned_gemm.json").write_text(json.dumps(t))
    monkeypatch.setattr(_build, "HERE", str(tmp_path))  # the digest reads the table next to the package
    assert _build.source_digest() != d0


def test_missing_explicit_table_raises(tmp_path):
    code = ("import sys; sys.path.insert(0, %r)\n"
            "from sdmi import kernels as K\n"
            "try:\n    K._tuned()\nexcept FileNotFoundError:\n    print('raised')\n") % PKG
    env = dict(os.environ, SDMI_TUNED_GEMM=str(tmp_path / "absent.json"))
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
    assert "raised" in out.stdout, out.stdout + out.stderr

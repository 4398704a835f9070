"""CPU checks of bench.py's arithmetic and fixtures (the GPU legs run on the
MI355X box): the DWT byte model against SURVEY.md 8(d)'s closed form, the
golden SHA-256 lookups the untimed validation uses, and the CLI parses."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)
import bench  # noqa: E402


@pytest.mark.parametrize("C,s,L,want", [(3, 1, 6, 22.99), (3, 2, 6, 25.99), (1, 2, 7, 8.666), (4, 1, 6, 30.66)])
def test_dwt_bytes_match_survey_formula(C, s, L, want):
    # B_dwt = C [s + 4 + (8/3)(1 - 4^-(L-1))] with 4-byte coefficients
    assert bench.dwt_bytes_per_px(C, s, L, 4) == pytest.approx(C * (s + 4 + 8 / 3 * (1 - 4.0 ** -(L - 1))), rel=1e-12)
    assert bench.dwt_bytes_per_px(C, s, L, 4) == pytest.approx(want, abs=0.01)


def test_golden_lookups_name_committed_fixtures():
    with open(os.path.join(ROOT, "tests", "golden", "golden.json")) as f:
        g = json.load(f)
    assert bench.golden_sha("c3") == g["c3_full"]["oracle_sha256"]
    assert bench.golden_sha("c4") == g["lossless"][0]["oracle_sha256"]
    c2 = [x for x in g["lossy"] if x["name"] == "c2_synth_rgb8_6000x4000"][0]
    assert bench.golden_sha("c2") == c2["oracle_sha256"]
    assert bench.golden_sha("nope") is None
    for k in ("c2", "c3", "c4"):
        assert len(bench.golden_sha(k)) == 64


def test_cli_parses():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--help"], capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0, r.stderr
    for flag in ("--gpus", "--steps", "--warmup", "--workload"):
        assert flag in r.stdout

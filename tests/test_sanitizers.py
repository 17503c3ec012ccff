"""SURVEY.md §5 "ASan/UBSan on the CPU transcription": the oracle's restatement of DPE.cu (every pass
type, edges / labels / geometric consistency / WEAK pixels on) and the host pipeline's image code
(JPEG decode, EdgeSegment and its restated OpenCV operations, the resamplers) run in executables
built with -fsanitize=address,undefined -fno-sanitize-recover=all; any report aborts them."""
import os
import subprocess

import numpy as np
import pytest
from PIL import Image

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=0", UBSAN_OPTIONS="print_stacktrace=1")


def _build(target, cwd):
    r = subprocess.run(["make", "-s", target], cwd=cwd, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]


@pytest.mark.timeout(900)
def test_oracle_under_asan_ubsan():
    _build("sanitize", os.path.join(ROOT, "oracle"))
    r = subprocess.run([os.path.join(ROOT, "oracle", "build", "oracle_sanitize")], capture_output=True, text=True,
                       timeout=300, env=ENV)
    assert r.returncode == 0, r.stderr[-4000:]
    assert "runtime error" not in r.stderr and r.stdout.count(" ok ") == 3, r.stdout + r.stderr[-2000:]


@pytest.mark.timeout(900)
def test_host_image_code_under_asan_ubsan(tmp_path):
    _build("sanitize-host", os.path.join(ROOT, "dpe-mvs_amd"))
    rng = np.random.default_rng(3)
    grey = (128 + 60 * np.sin(np.arange(97)[:, None] / 6.0) * np.cos(np.arange(131)[None, :] / 9.0)).astype(np.uint8)
    grey[20:40, 30:90] = 200
    gp, cp = str(tmp_path / "g.jpg"), str(tmp_path / "c.jpg")
    Image.fromarray(grey, mode="L").save(gp, quality=90)
    Image.fromarray(rng.integers(0, 256, (37, 53, 3), dtype=np.uint8), mode="RGB").save(cp, quality=85, subsampling=2)
    r = subprocess.run([os.path.join(ROOT, "dpe-mvs_amd", "bin", "host_sanitize"), gp, cp], capture_output=True,
                       text=True, timeout=300, env=ENV)
    assert r.returncode == 0, r.stderr[-4000:]
    assert "runtime error" not in r.stderr and "host sanitize ok" in r.stdout, r.stdout + r.stderr[-2000:]

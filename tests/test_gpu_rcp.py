"""The 3-op reciprocal used in the NCC tap loops (device_math.h d_rcp_fast) is bit-identical to IEEE
1.0f / z for every float with biased exponent in [1, 252], both signs: exhaustive check on the GPU
(tools/rcp_check.hip, 2^23 mantissas x 256 exponents x 2 signs)."""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
def test_fast_rcp_exhaustive(tmp_path):
    exe = str(tmp_path / "rcp_check")
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-ffp-contract=off",
                    os.path.join(ROOT, "tools", "rcp_check.hip"), "-o", exe], check=True, capture_output=True)
    out = subprocess.run([exe], check=True, capture_output=True, text=True, timeout=300).stdout
    m = re.search(r"biased exponent in \[1, 252\]: (\d+)", out)
    assert m and int(m.group(1)) == 0, out

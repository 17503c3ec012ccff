"""TEST INFRASTRUCTURE: builds oracle/rcp_gfx950.bin.xz, the oracle's model of gfx950's v_rcp_f32
(restatement choice 8: the tap reciprocal, oracle_math.h o_rcp_hw), from a dump of the instruction
over every mantissa at biased exponent 127 (tools/rcp_dump.hip run on an MI355X, which also checks
that the result at every other exponent 1..252 and either sign is this one scaled):

    python oracle/make_rcp_table.py gpurun_out/rcp127.bin

Code per mantissa m of z = 1.m: bits(v_rcp_f32(z)) - bits(RN(1/z)) + 1, in {0, 1, 2}; four codes per
byte (code of m at bits 2 (m & 3)), 2 MiB, stored lzma-compressed (~105 KB).  tests/test_gpu_rcp.py
re-checks the model against the device instruction on every -m gpu run."""
import lzma
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))


def main(dump):
    r = np.fromfile(dump, dtype=np.uint32)
    assert r.size == 1 << 23, r.size
    m = np.arange(1 << 23, dtype=np.uint32)
    z = (np.uint32(127 << 23) | m).view(np.float32)
    ieee = (np.float32(1.0) / z).astype(np.float32).view(np.uint32)
    d = r.astype(np.int64) - ieee.astype(np.int64)
    assert d.min() >= -1 and d.max() <= 1, (d.min(), d.max())
    c = (d + 1).astype(np.uint8)
    packed = (c[0::4] | (c[1::4] << 2) | (c[2::4] << 4) | (c[3::4] << 6)).astype(np.uint8).tobytes()
    out = os.path.join(HERE, "rcp_gfx950.bin.xz")
    with open(out, "wb") as f:
        f.write(lzma.compress(packed, preset=9 | lzma.PRESET_EXTREME))
    print(f"{out}: -1 ulp {int((d == -1).sum())}, +1 ulp {int((d == 1).sum())} of 2^23 mantissas")


if __name__ == "__main__":
    main(sys.argv[1])

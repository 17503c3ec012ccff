"""Rates of the coarse pyramid levels of the schedule (bench.coarse_level_pass: 800x600 and 1344x896
REFINE_ITER + geom passes on INTER_LINEAR-downscaled images) for the library DPE_MVS_LIB names.
Usage: DPE_MVS_LIB=lib/variants/x.so python tools/levels.py"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "dpe-mvs_amd"))
import torch  # noqa: E402
torch.cuda.set_device(0)
import bench  # noqa: E402
from DPE_MVS import _abi, native, synthetic  # noqa: E402

sp = torch.cuda.Stream()
out = {"lib": os.path.basename(native.LIB_PATH)}
for Wl, Hl in ((1600, 1200), (2688, 1792)):
    out[f"{Wl // 2}x{Hl // 2}"] = bench.coarse_level_pass(native, _abi, synthetic, 0, sp.cuda_stream, Wl, Hl)
print(json.dumps(out), flush=True)

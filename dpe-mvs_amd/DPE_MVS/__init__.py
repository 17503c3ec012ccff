"""DPE_MVS — MI355X-native PatchMatch multi-view stereo (drop-in for DPE-MVS's depth/normal path).

Submodules:
  native     ctypes binding of the HIP C-ABI library (lib/libdpe_mvs.so): one PatchMatch pass
  synthetic  synthetic pinhole scenes with ground truth (tests and benchmark inputs)
  _abi       ctypes mirror of include/dpe_mvs.h
"""
from __future__ import annotations

__all__ = ["native", "synthetic"]

"""DPE_MVS — MI355X-native PatchMatch multi-view stereo (drop-in for DPE-MVS's depth/normal path).

Submodules:
  native     ctypes binding of the HIP C-ABI library (lib/libdpe_mvs.so): one PatchMatch pass
  synthetic  synthetic pinhole scenes with ground truth (tests and benchmark inputs)
  _abi       ctypes mirror of include/dpe_mvs.h
  pipeline   the host pipeline (RunDPEPipeline / ProcessProblem) over the C-ABI, dpe_mvs()
"""
from __future__ import annotations


def dpe_mvs(dense_folder: str, gpu_index: int = 0, verbose: bool = True, fusion: bool = False, viz: bool = False,
            depth: bool = True, normal: bool = False, weak: bool = False, edge: bool = False) -> int:
    """Run the DPE-MVS pipeline from Python (same signature as the reference's DPE_MVS.dpe_mvs)."""
    from .pipeline import dpe_mvs as _run
    return _run(dense_folder, gpu_index, verbose, fusion, viz, depth, normal, weak, edge)


__all__ = ["dpe_mvs", "native", "synthetic", "pipeline"]

"""DPE_MVS — MI355X-native PatchMatch multi-view stereo (drop-in for DPE-MVS's depth/normal path).

Submodules:
  native     ctypes binding of the HIP C-ABI library (lib/libdpe_mvs.so): one PatchMatch pass
  synthetic  synthetic pinhole scenes with ground truth (tests and benchmark inputs)
  _abi       ctypes mirror of include/dpe_mvs.h
  pipeline   ctypes side of the C++ host pipeline (lib/libdpe_host.so): multi-rank runs, hooks
  _dpe       pybind11 module of the C++ host pipeline (built by make): dpe_mvs()
  colmap2mvsnet  COLMAP sparse model -> dense_folder converter (python -m DPE_MVS.colmap2mvsnet)
"""
from __future__ import annotations


def dpe_mvs(dense_folder: str, gpu_index: int = 0, verbose: bool = True, fusion: bool = False, viz: bool = False,
            depth: bool = True, normal: bool = False, weak: bool = False, edge: bool = False) -> int:
    """Run the DPE-MVS pipeline from Python (same signature as the reference's DPE_MVS.dpe_mvs,
    src/DPE_MVS/__init__.py:6-17): the C++ host pipeline through the pybind11 module `_dpe`."""
    from ._dpe import dpe_mvs as _native
    return _native(dense_folder, gpu_index, verbose, fusion, viz, depth, normal, weak, edge)


__all__ = ["dpe_mvs", "native", "synthetic", "pipeline"]

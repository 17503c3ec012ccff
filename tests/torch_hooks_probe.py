"""Driven by tests/test_pipeline.py::test_gpu_torch_nccl_hooks_single_rank (one GPU): the torch
"nccl" (RCCL) all-gather hooks of DPE_MVS.pipeline -- the device hook on __cuda_array_interface__
views of the library's own HBM buffers and the host hook -- called exactly as the C++ pipeline calls
them, in a one-rank process group.  What one GPU cannot check is the multi-rank transport itself."""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dpe-mvs_amd"))
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402
from DPE_MVS import native, pipeline  # noqa: E402


def main():
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    lib = native.load_library()
    lib.dpe_device_buffer.argtypes = [C.c_void_p, C.c_int, C.c_size_t]
    lib.dpe_device_buffer.restype = C.c_void_p
    lib.dpe_device_copy.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
    ctx = lib.dpe_create(0)
    try:
        n = 123457
        send = lib.dpe_device_buffer(ctx, 0, n)
        recv = lib.dpe_device_buffer(ctx, 1, n)
        assert send and recv
        a = np.random.default_rng(7).standard_normal(n).astype(np.float32)
        assert lib.dpe_device_copy(ctx, send, a.ctypes.data, a.nbytes, 0) == 0
        assert lib.dpe_device_copy(ctx, recv, np.zeros(n, np.float32).ctypes.data, a.nbytes, 0) == 0
        dev = pipeline._torch_allgather_device(dist)
        assert dev(None, send, n, recv) == 0
        b = np.empty(n, np.float32)
        assert lib.dpe_device_copy(ctx, b.ctypes.data, recv, b.nbytes, 1) == 0
        assert np.array_equal(a.view(np.uint32), b.view(np.uint32)), "device hook"
        host = pipeline._torch_allgather(dist)
        c = np.empty(n, np.float32)
        fp = C.POINTER(C.c_float)
        assert host(None, a.ctypes.data_as(fp), n, c.ctypes.data_as(fp)) == 0
        assert np.array_equal(a.view(np.uint32), c.view(np.uint32)), "host hook"
        print("HOOKS_OK", flush=True)
    finally:
        lib.dpe_destroy(ctx)
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

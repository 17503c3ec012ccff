"""Python launcher with the positional arguments of the reference's `DPE` binary (main.cpp:602-635);
the native command line is dpe-mvs_amd/bin/dpe (same arguments, RCCL across ranks):

    python -m DPE_MVS dense_folder [gpu_index] [verbose] [viz] [fusion] [depth] [normal] [weak] [edge]

Multi-GPU (one process per GPU, reference images sharded, depth maps all-gathered over RCCL):

    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 -m DPE_MVS dense_folder
"""
from __future__ import annotations

import os
import sys


def main(argv: list) -> int:
    if len(argv) < 2:
        print("USAGE: DPE dense_folder", file=sys.stderr)
        return 1
    a = [int(x) for x in argv[2:]]
    opt = lambda i, d: a[i] if len(a) > i else d
    gpu_index, verbose, viz, fusion = opt(0, 0), bool(opt(1, 1)), bool(opt(2, 0)), bool(opt(3, 0))
    depth, normal, weak, edge = bool(opt(4, 1)), bool(opt(5, 0)), bool(opt(6, 0)), bool(opt(7, 0))
    from . import pipeline
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world > 1:
        import torch
        import torch.distributed as dist
        local = int(os.environ.get("LOCAL_RANK", "0"))
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        try:
            return pipeline.run_dpe_pipeline(argv[1], local, verbose, fusion, viz, depth, normal, weak, edge, dist=dist)
        finally:
            dist.destroy_process_group()
    return pipeline.dpe_mvs(argv[1], gpu_index, verbose, fusion, viz, depth, normal, weak, edge)


if __name__ == "__main__":
    sys.exit(main(sys.argv))

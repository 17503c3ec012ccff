"""HBM-resident pipeline state (include/dpe_mvs.h dpe_state_* / dpe_pm_stage_resident): with the HIP
library as the pass runner the host pipeline keeps every image's depth / normal / weak / selected-view
maps on the device between passes (the reference's depths.dmb / normals.dmb / weak.bin /
selected_views.bin round trip, main.cpp:439-446, DPE.cpp:826-911), rescales priors and source depths
there and applies ProcessProblem's epilogue there.  The host-buffer path (any custom runner, here the
oracle) is the checker: outputs must be byte-identical for both schedules, with the intermediate maps
written, and with two ranks exchanging depth maps between passes."""
import os
import shutil
import socket

import numpy as np
import pytest

from DPE_MVS import _abi, pipeline, synthetic
from test_pipeline import oracle_runner, _copy, OUTS

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dense4(tmp_path_factory):
    d = str(tmp_path_factory.mktemp("dense4r"))
    synthetic.write_dense_folder(d, 64, 48, 4)
    return d


def _outputs(folder, n, files=("depth.npy", "normal.npy", "weak.npy")):
    return {(i, f): np.load(os.path.join(folder, "DPE", f"{i:08d}", f)) for i in range(n) for f in files}


def _same(a, b):
    for k in a:
        assert a[k].dtype == b[k].dtype and a[k].tobytes() == b[k].tobytes(), k


@pytest.mark.parametrize("schedule", ["reference", "jacobi"])
def test_resident_pipeline_matches_host_path(tmp_path, dense4, schedule):
    a = _copy(dense4, tmp_path, "hip")
    b = _copy(dense4, tmp_path, "cpu")
    assert pipeline.run_dpe_pipeline(a, schedule=schedule, normal=True, weak=True, verbose=False) == 0
    assert pipeline.run_dpe_pipeline(b, runner=oracle_runner(), schedule=schedule, normal=True, weak=True,
                                     verbose=False) == 0
    _same(_outputs(a, 4), _outputs(b, 4))


def test_resident_keep_intermediate_writes_the_reference_maps(tmp_path, dense4):
    a = _copy(dense4, tmp_path, "hip")
    b = _copy(dense4, tmp_path, "cpu")
    assert pipeline.run_dpe_pipeline(a, normal=True, weak=True, verbose=False, keep_intermediate=True) == 0
    assert pipeline.run_dpe_pipeline(b, runner=oracle_runner(), normal=True, weak=True, verbose=False,
                                     keep_intermediate=True) == 0
    _same(_outputs(a, 4), _outputs(b, 4))
    for i in range(4):
        for f in ("depths.dmb", "normals.dmb", "weak.bin", "selected_views.bin"):
            x = pipeline.read_bin_mat(os.path.join(a, "DPE", f"{i:08d}", f))
            y = pipeline.read_bin_mat(os.path.join(b, "DPE", f"{i:08d}", f))
            assert x.dtype == y.dtype and x.tobytes() == y.tobytes(), (i, f)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _rank_main(rank, world, port, folder):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:   # both ranks on GPU 0; gloo -> the host all-gather hook around the device export / import
        assert pipeline.run_dpe_pipeline(folder, normal=True, weak=True, verbose=False, dist=dist) == 0
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(600)
def test_resident_two_ranks_match_one_rank_jacobi(tmp_path, dense4):
    import torch.multiprocessing as mp
    one = _copy(dense4, tmp_path, "one")
    two = _copy(dense4, tmp_path, "two")
    assert pipeline.run_dpe_pipeline(one, runner=oracle_runner(), schedule="jacobi", normal=True, weak=True,
                                     verbose=False) == 0
    mp.start_processes(_rank_main, args=(2, _free_port(), two), nprocs=2, join=True, start_method="spawn")
    _same(_outputs(one, 4), _outputs(two, 4))


def _rank_main_devhook(rank, world, port, folder, fault, q):
    """A rank whose device all-gather hook is a host hop over gloo (so the device exchange path of
    host/pipeline.cpp -- dsend packing, the import offsets r * cnt + k * per -- runs on one GPU).
    `fault` ("before:R" / "after:R", DPE_FAULT_INJECT): rank R fails locally just before the first
    resident exchange's status all-gather, or just after its depth all-gather."""
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    if fault:
        os.environ["DPE_FAULT_INJECT"] = fault
    dist.init_process_group("gloo", rank=rank, world_size=world)
    calls = [0]

    def hook(send, count, recv):
        calls[0] += 1
        s = torch.as_tensor(pipeline._DeviceArray(send, count), device="cuda")
        r = torch.as_tensor(pipeline._DeviceArray(recv, world * count), device="cuda")
        out = torch.empty(world * count, dtype=torch.float32)
        dist.all_gather_into_tensor(out, s.cpu())
        r.copy_(out.to("cuda"))
        torch.cuda.synchronize()
        return 0
    try:
        pipeline.run_dpe_pipeline(folder, normal=True, weak=True, verbose=False, dist=dist, allgather_device=hook)
        q.put((rank, "ok", calls[0]))
    except pipeline.PipelineError as e:
        q.put((rank, str(e), calls[0]))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(600)
@pytest.mark.parametrize("fault", ["", "before:1", "after:1"])
def test_resident_device_hook_path(tmp_path, dense4, fault):
    import torch.multiprocessing as mp
    one = _copy(dense4, tmp_path, "one")
    two = _copy(dense4, tmp_path, "two")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    mp.start_processes(_rank_main_devhook, args=(2, _free_port(), two, fault, q), nprocs=2, join=True,
                       start_method="spawn")
    got = {r: (msg, n) for r, msg, n in (q.get(timeout=10) for _ in range(2))}
    if not fault:
        assert all(n > 0 for _, n in got.values()), got          # the device hook carried the exchange
        assert all(msg == "ok" for msg, _ in got.values()), got
        assert pipeline.run_dpe_pipeline(one, runner=oracle_runner(), schedule="jacobi", normal=True, weak=True,
                                         verbose=False) == 0
        _same(_outputs(one, 4), _outputs(two, 4))
    elif fault.startswith("before"):
        # every rank ends at the first exchange's status all-gather, before any depth all-gather
        assert got[0] == ("rank 1 failed", 0), got
        assert got[1] == ("injected fault before the exchange", 0), got
    else:
        # rank 1 fails after the first depth all-gather, which every rank completed; the others are
        # not left behind: every rank ends at the next exchange's status all-gather
        assert got[0] == ("rank 1 failed", 1), got
        assert got[1] == ("injected fault after the exchange", 1), got

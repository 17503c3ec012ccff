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

"""Where RunFusion's time goes at BASELINE configs[4] (bench.py pipeline_config5): runs the config-5
pipeline once on GPU 0 with DPE_FUSION_PROFILE=1, which prints the seconds spent waiting for the
candidate copies, in the parallel angle / weight terms and in the serial walk (host/fusion.cpp).
Usage: python tools/fusion_prof.py [n_images] [width] [height]"""
import os
import shutil
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dpe-mvs_amd"))
os.environ["DPE_FUSION_PROFILE"] = "1"
import torch  # noqa: E402,F401
from DPE_MVS import pipeline, synthetic  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 32
W = int(sys.argv[2]) if len(sys.argv) > 2 else 1920
H = int(sys.argv[3]) if len(sys.argv) > 3 else 1080
folder = f"/tmp/dpe_fusion_prof_{os.getpid()}"
try:
    sc = synthetic.make_scene(W, H, n)
    synthetic.write_dense_folder(folder, W, H, n, max_src=min(31, n - 1), with_edges=False, scene=sc)
    del sc
    t0 = time.perf_counter()
    pipeline.run_dpe_pipeline(folder, gpu_index=0, verbose=False, fusion=True)
    import ctypes
    ph = (ctypes.c_double * 8)()
    pipeline.lib().dpe_pipeline_last_timings(ph, 8)
    print(f"{n} x {W}x{H}: wall {time.perf_counter() - t0:.2f} s, passes {ph[6]:.2f} s, fusion {ph[7]:.2f} s", flush=True)
finally:
    shutil.rmtree(folder, ignore_errors=True)

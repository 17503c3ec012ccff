"""Loads the committed golden fixtures (tests/golden/*.npz) back into pass inputs."""
import ast
import glob
import os

import numpy as np

from DPE_MVS import _abi

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def names():
    return sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLDEN, "*.npz")))


def load(name):
    z = np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)
    cams = []
    for row in z["cams"]:
        c = _abi.DpeCamera()
        for i in range(9):
            c.K[i] = float(row[i]); c.R[i] = float(row[9 + i])
        for i in range(3):
            c.t[i] = float(row[18 + i]); c.c[i] = float(row[21 + i])
        c.height, c.width = int(row[24]), int(row[25])
        c.depth_min, c.depth_max = float(row[26]), float(row[27])
        cams.append(c)
    p = _abi.DpePatchMatchParams()
    for k, v in ast.literal_eval(str(z["params"][0])).items():
        setattr(p, k, v)
    images = [im.astype(np.float32) for im in z["images"]]
    depths = None
    if z["depths"].size:
        depths = [None] + [d for d in z["depths"][1:]]
    inp = dict(images=images, cams=cams, depths=depths, edge=z["edge"], edge_low=z["edge_low"], label=z["label"],
               params=p, seed=int(z["seed"]), pass_salt=int(z["pass_salt"]))
    st = dict(planes=z["in_planes"], weak=z["in_weak"], sel=z["in_sel"])
    exp = dict(planes=z["out_planes"], weak=z["out_weak"], sel=z["out_sel"], costs=z["out_costs"])
    return inp, st, exp


def bits_equal(a, b):
    a = np.ascontiguousarray(a); b = np.ascontiguousarray(b)
    if a.dtype == np.float32:
        return np.array_equal(a.view(np.uint32), b.view(np.uint32))
    return np.array_equal(a, b)

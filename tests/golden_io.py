"""Load committed golden fixtures (inputs + expected oracle outputs)."""
import os

import numpy as np

from plba.synth import Graph

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(cfg):
    path = os.path.join(GOLDEN, f"{cfg}.npz")
    g = Graph.load(path)
    with np.load(path, allow_pickle=False) as z:
        out = {k[4:]: z[k] for k in z.files if k.startswith("out_")}
    return g, out

"""Helpers to enumerate and load the committed golden fixtures (data only)."""
import glob
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def cases():
    out = []
    for meta_path in sorted(glob.glob(os.path.join(GOLDEN, "*", "K*_s*.json"))):
        case_dir = os.path.dirname(meta_path)
        name = os.path.basename(meta_path)[:-5]
        out.append((os.path.basename(case_dir), name))
    return out


def load(case, name):
    d = os.path.join(GOLDEN, case)
    with open(os.path.join(d, name + ".json")) as f:
        meta = json.load(f)
    vec = np.load(os.path.join(d, name + ".npz"), allow_pickle=False)
    return meta, vec, os.path.join(d, "train.dat"), os.path.join(d, "test.dat")

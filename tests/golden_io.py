"""Loader for the committed sklearn golden vectors (tests/golden/*.npz, made by make_golden.py)."""
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def names():
    with open(os.path.join(GOLDEN, "MANIFEST.json")) as f:
        return sorted(json.load(f)["cases"])


def load(name):
    z = np.load(os.path.join(GOLDEN, f"{name}.npz"), allow_pickle=False)
    case = {k: z[k] for k in z.files}
    case["kwargs"] = json.loads(str(case["kwargs"]))
    case["n_iter"] = int(case["n_iter"])
    return case


def init_names():
    with open(os.path.join(GOLDEN, "MANIFEST.json")) as f:
        return sorted(json.load(f)["init_cases"])


def load_init(name):
    """X, W, H = sklearn's _initialize_nmf(X, **kwargs) (make_golden.py:init_cases)."""
    z = np.load(os.path.join(GOLDEN, f"{name}.npz"), allow_pickle=False)
    case = {k: z[k] for k in z.files}
    case["kwargs"] = json.loads(str(case["kwargs"]))
    return case


def rel_fro(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    den = np.linalg.norm(b)
    return float(np.linalg.norm(a - b) / (den if den > 0 else 1.0))

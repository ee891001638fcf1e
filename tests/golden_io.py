"""Loading helpers for tests/golden/nav_goldens.json.gz (reference outputs)."""
from __future__ import annotations

import functools
import gzip
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "nav_goldens.json.gz")


@functools.lru_cache(maxsize=1)
def load_goldens() -> dict:
    with gzip.open(GOLDEN, "rt") as f:
        return json.load(f)


def cells_of(frame: dict) -> np.ndarray:
    return np.array([[ch == "1" for ch in row] for row in frame["cells"]], dtype=bool)


def unhex(v):
    """Golden scalar -> python value (int for 'iN', float for hex, None)."""
    if v is None:
        return None
    if isinstance(v, str) and v.startswith("i"):
        return int(v[1:])
    if v == "inf":
        return float("inf")
    return float.fromhex(v)


def key_tuple(k):
    return ((k[0], k[1]), (k[2], k[3]))

"""Loader for the reference-generated fixtures in tests/golden/ (see gen_golden.py)."""
import hashlib
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def manifest():
    with open(os.path.join(GOLDEN, "manifest.json")) as f:
        return json.load(f)


def kat():
    with open(os.path.join(GOLDEN, "kat.json")) as f:
        return json.load(f)


def rgb(entry):
    b = open(os.path.join(GOLDEN, entry["rgb_file"]), "rb").read()
    return np.frombuffer(b, np.uint8).reshape(entry["H"], entry["W"], 3)


def sums(entry):
    if "sums_file" not in entry:
        return None
    b = open(os.path.join(GOLDEN, entry["sums_file"]), "rb").read()
    return np.frombuffer(b, "<f8").reshape(entry["H"], entry["W"], 3)


def sha(arr) -> str:
    return hashlib.sha256(np.ascontiguousarray(arr).tobytes()).hexdigest()

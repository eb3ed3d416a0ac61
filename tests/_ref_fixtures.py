"""Reference-owned fixtures for the CPU suite: the copies vendored under tests/fixtures (tools/vendor_fixtures.py),
falling back to the reference tree when a copy is missing. Numeric literals of reference unit tests come from the
vendored JSON extracts (tests/fixtures/java/<Test>.json), never from parsing Java at test time."""
import json
import os

import torch

FIX = os.path.join(os.path.dirname(os.path.abspath(__file__)), "fixtures")
REF = "/root/reference"


def path(rel):
    """Vendored copy of reference file / directory ``rel`` (relative to the reference root), else the original."""
    v = os.path.join(FIX, rel)
    return v if os.path.exists(v) else os.path.join(REF, rel)


def exists(rel):
    return os.path.exists(path(rel))


def _java(test_name):
    with open(os.path.join(FIX, "java", test_name + ".json")) as fh:
        return json.load(fh)


def _tensor(a):
    return torch.tensor(a["values"], dtype=torch.float64).reshape(a["shape"])


def java_arrays(test_name, after):
    """Every Nd4j.create(double[], int[]) literal after the declaration ``after`` ("public void testX" /
    "public INDArray getContainedData": the method name is what counts)."""
    d = _java(test_name)
    name = after.split()[-1]
    pos = d["declarations"][name]
    return [_tensor(a) for a in d["arrays"] if a["pos"] > pos]


def java_named(test_name, var):
    """The first literal assigned to variable ``var``."""
    for a in _java(test_name)["arrays"]:
        if a["name"] == var:
            return _tensor(a)
    raise KeyError(var)

"""Kernel-choice database (ops/tunedb.py): record -> save -> reload round trip with the value types the autotuners
store (GEMM (cfg, splits) tuples, conv variant ints, weight-gradient engine tuples, 1x1 GEMM-vs-conv booleans),
merging into an existing file, schema-version isolation and the off switch."""
import json

import pytest
import torch

from deeplearning4j_amd.ops import tunedb


@pytest.fixture
def fresh(monkeypatch):
    monkeypatch.setattr(tunedb, "_db", None)
    monkeypatch.setattr(tunedb, "_recorded", {})
    monkeypatch.setattr(tunedb, "_path_used", None)
    yield monkeypatch


def test_round_trip_types(tmp_path, fresh):
    gk = (4096, 768, 3072, 1, 1, 1, True, False, True, True)
    ck = ("fwd", (64, 56, 56, 64, 64, 3, 3, 1, 1, 1, 1, 1, 1, 56, 56), False, True, torch.bfloat16)
    wk = ((64, 56, 56, 64, 64, 3, 3, 1, 1, 1, 1, 1, 1, 56, 56), False, torch.bfloat16)
    tunedb.record("gemm", gk, (3, 2))
    tunedb.record("conv_v3", ck, 1)
    tunedb.record("conv_wrw", wk, ("halo", 1, 16))
    tunedb.record("conv_1x1", ("dx", (8, 64), False), True)
    p = tmp_path / "gfx950.json"
    assert tunedb.save(str(p), arch="gfx950") == 4
    data = json.loads(p.read_text())
    assert data["version"] == tunedb.VERSION and data["arch"] == "gfx950"
    fresh.setattr(tunedb, "_db", None)
    fresh.setenv("DL4J_AMD_TUNE_DB", str(p))
    assert tunedb.lookup("gemm", gk) == (3, 2)
    assert tunedb.lookup("conv_v3", ck) == 1
    assert tunedb.lookup("conv_wrw", wk) == ("halo", 1, 16)
    assert tunedb.lookup("conv_1x1", ("dx", (8, 64), False)) is True
    assert tunedb.lookup("gemm", gk[:-1]) is None
    assert tunedb.loaded_from() == str(p)


def test_save_merges_existing_and_ignores_other_versions(tmp_path, fresh):
    p = tmp_path / "db.json"
    tunedb.record("gemm", (1, 2, 3), (0, 1))
    tunedb.save(str(p))
    fresh.setattr(tunedb, "_recorded", {})
    tunedb.record("gemm", (4, 5, 6), (2, 3))
    assert tunedb.save(str(p)) == 2
    fresh.setenv("DL4J_AMD_TUNE_DB", str(p))
    fresh.setattr(tunedb, "_db", None)
    assert tunedb.lookup("gemm", (1, 2, 3)) == (0, 1) and tunedb.lookup("gemm", (4, 5, 6)) == (2, 3)
    old = json.loads(p.read_text())
    old["version"] = tunedb.VERSION - 1
    p.write_text(json.dumps(old))
    fresh.setattr(tunedb, "_db", None)
    assert tunedb.lookup("gemm", (1, 2, 3)) is None


def test_off_switch_and_reps(tmp_path, fresh):
    p = tmp_path / "db.json"
    tunedb.record("gemm", (7,), (5, 1))
    tunedb.save(str(p))
    fresh.setenv("DL4J_AMD_TUNE_DB", "off")
    fresh.setattr(tunedb, "_db", None)
    assert tunedb.lookup("gemm", (7,)) is None
    fresh.setenv("DL4J_AMD_TUNE_REPS", "9")
    assert tunedb.reps(3) == 9
    fresh.setenv("DL4J_AMD_TUNE_REPS", "1")
    assert tunedb.reps(3) == 3


def test_cu_count_mismatch_ignores_file_and_forget(tmp_path, fresh):
    """A file timed on a device with another compute-unit count is ignored; a refused entry is dropped by forget()."""
    p = tmp_path / "gfx950.json"
    p.write_text(json.dumps({"version": tunedb.VERSION, "arch": "gfx950", "cus": 256,
                             "tables": {"gemm": {repr((1, 2, 3)): [3, 2]}}}))
    fresh.setenv("DL4J_AMD_TUNE_DB", str(p))
    fresh.setattr(tunedb, "_cus", lambda: 304)
    assert tunedb.lookup("gemm", (1, 2, 3)) is None
    fresh.setattr(tunedb, "_db", None)
    fresh.setattr(tunedb, "_cus", lambda: 256)
    assert tunedb.lookup("gemm", (1, 2, 3)) == (3, 2)
    tunedb.forget("gemm", (1, 2, 3))
    assert tunedb.lookup("gemm", (1, 2, 3)) is None
    fresh.setattr(tunedb, "_db", None)
    fresh.setattr(tunedb, "_cus", lambda: None)       # no device (CPU): the file is used as is
    assert tunedb.lookup("gemm", (1, 2, 3)) == (3, 2)

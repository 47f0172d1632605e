"""bench.py's host-side accounting (no GPU): the byte models of SURVEY.md
8(d), the measured-traffic roofline and its refusal of a PMC record taken on
a different library build, and the host-core count the CPU baseline reports."""
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402

REDDIT = dict(n=232965, nnz=23446803, F=602)


def test_byte_models_reddit():
    # the figures DESIGN.md 5 quotes per hop at the Reddit shape
    assert bench.gather_model_bytes(**REDDIT) == 57209387632
    assert bench.compulsory_bytes(**REDDIT) == 1310465728


def test_roofline_refuses_traffic_of_another_build():
    rec = bench.roofline("reddit", REDDIT["n"], REDDIT["nnz"], REDDIT["F"], 4.65, 4.45, 4.6,
                         "0" * 64, "one hop", "spmm_rows_kernel")
    assert rec["traffic"] is None and "refused" in rec["traffic_source"]
    assert rec["frac"] == pytest.approx(rec["compulsory_frac"])
    assert rec["hub_tail_ms"] == pytest.approx(0.15)


@pytest.mark.parametrize("shape", ["reddit", "rmat"])
def test_roofline_uses_matching_pmc_record(shape):
    path = os.path.join(ROOT, "profiles", f"pmc_{shape}.json")
    pmc = json.load(open(path))
    pmc_sha = pmc["lib_sha256"]
    G = int(pmc.get("dispatches_per_launch", 1))
    traffic, src = bench.load_traffic(shape, pmc_sha, G)
    assert traffic is not None and traffic["hbm_bytes_per_launch"] > 0
    # a record of another schedule (column-group dispatches per hop) is refused
    other, why = bench.load_traffic(shape, pmc_sha, G + 1)
    assert other is None and "refused" in why
    ms = float(pmc["kernel_ms"])  # the hop time the counters were taken over
    rec = bench.roofline(shape, REDDIT["n"], REDDIT["nnz"], REDDIT["F"], ms, ms, None,
                         pmc_sha, "one hop", "spmm_rows_kernel", G)
    t = ms * 1e-3
    assert rec["traffic"] == traffic["hbm_bytes_per_launch"]
    assert rec["frac"] == pytest.approx(rec["traffic"] / t / 1e9 / bench.HBM_PEAK_GBS)
    assert 0 < rec["frac"] <= 1.0


def test_host_cores_positive():
    n, how = bench.host_cores()
    assert n >= 1 and "sched_getaffinity" in how


def test_self_launch_refuses_more_ranks_than_gpus(monkeypatch, capsys):
    """--gpus N over RCCL with fewer visible GPUs: refused before any rank is
    started (exit status 2), without touching the GPU runtime."""
    import argparse
    monkeypatch.setattr(bench.torch.cuda, "device_count", lambda: 1)
    args = argparse.Namespace(gpus=4, dist_backend="nccl")
    assert bench.self_launch(args) == 2
    assert "needs 4 GPUs" in capsys.readouterr().err


def test_host_cols_ascending():
    """The host check that turns column groups on for from_host_arrays CSRs:
    strictly ascending columns within every row (empty rows allowed)."""
    import numpy as np
    from sgc_amd.propagate import _host_cols_ascending as asc
    assert asc(np.array([0, 2, 2, 5]), np.array([1, 3, 0, 2, 9]))
    assert not asc(np.array([0, 2, 2, 5]), np.array([1, 3, 0, 2, 2]))  # duplicate
    assert not asc(np.array([0, 2, 5]), np.array([3, 1, 0, 2, 9]))     # descending
    assert asc(np.array([0, 0, 0]), np.array([], dtype=np.int32))
    assert asc(np.array([0, 1, 2]), np.array([5, 0]))                    # one per row

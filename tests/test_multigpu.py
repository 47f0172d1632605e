"""sgc_precompute across processes behind the reference's own call
(sgc_amd.multigpu; reference reddit.py:43 -> utils.py:92-97), on CPU over gloo.

Each worker is started the way torchrun starts a rank -- RANK / WORLD_SIZE /
LOCAL_RANK / MASTER_* in its environment, no process group yet -- and calls
the unchanged `sgc_precompute(features, adj, K)`: the first call initialises
the group from that environment and the hops run partitioned.  Every rank's
X_K must equal the reference's (the golden vectors) bit for bit, for each
partition.  The GPU versions (RCCL, the one-GPU gloo rehearsal, the native
multi-device engine) are in tests/test_gpu_multigpu.py.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _torchrun_like_worker(rank, world, port, case, K, partition, q, env=None, calls=2):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      LOCAL_WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port), SGC_AMD_PARTITION=partition, **(env or {}))
    import torch.distributed as dist
    from sgc_amd import multigpu
    from sgc_amd.utils import sgc_precompute
    try:
        n = int(case["n"])
        adj = torch.sparse_coo_tensor(torch.from_numpy(np.stack([case["rows"], case["cols"]])),
                                      torch.from_numpy(case["vals"]), (n, n))
        X = torch.from_numpy(case["X"])
        outs, props = [], []
        for _ in range(calls):  # later calls: cached partition, buffers reused
            before = multigpu.PROPAGATIONS[0]
            out, secs = sgc_precompute(X, adj, K)
            props.append(multigpu.PROPAGATIONS[0] - before)
            outs.append(out)
        rec = multigpu.auto_choice(adj._sgc_amd_csr[1], dist.group.WORLD, X.shape[1], K)
        from sgc_amd.distributed import SETUP_SECONDS
        q.put((rank, outs[0].numpy().copy(), all(torch.equal(outs[0], o) for o in outs),
               dist.get_world_size(), secs >= 0, None if rec is None else dict(rec), props,
               dict(SETUP_SECONDS)))
    finally:
        import torch.distributed as dist2
        if dist2.is_initialized():
            dist2.destroy_process_group()


def _run_world(case, world, K, partition, env=None, calls=2):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_torchrun_like_worker,
                         args=(r, world, port, case, K, partition, q, env, calls))
             for r in range(world)]
    for p in procs:
        p.start()
    got = dict((r, rest) for r, *rest in (q.get(timeout=180) for _ in range(world)))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = case[f"Y{K}"]
    for r in range(world):
        out, stable, ws, timed = got[r][:4]
        assert ws == world and stable and timed
        assert out.shape == want.shape
        assert np.array_equal(out.view(np.uint32), want.view(np.uint32)), (partition, r)
    return got


@pytest.mark.parametrize("world,name,K,partition", [
    (2, "norm_n48_F602", 2, "features"), (3, "hub1000_F65", 2, "features"),
    (3, "raw_unsorted_dups_F7", 3, "features"), (2, "special_values_F11", 2, "rows"),
    (2, "norm_n48_F65", 2, "rows"), (3, "norm_n48_F130", 2, "rows"),
    (2, "hub1000_F130", 2, "cyclic"), (4, "norm_n48_F65", 3, "cyclic"),
    (2, "isolated_F17", 1, "features"), (2, "norm_n48_F602", 2, "lines"),
    (3, "hub1000_F130", 2, "lines"), (4, "norm_n48_F602", 2, "auto"),
    (2, "norm_n48_F602", 2, "replicate"), (3, "hub1000_F130", 2, "replicate"),
    (2, "hub1000_F130", 2, "auto"), (3, "raw_unsorted_dups_F7", 2, "auto")])
def test_sgc_precompute_under_torchrun_env(tiny_cases, world, name, K, partition):
    from sgc_amd.multigpu import rule_choice
    case = tiny_cases[name]
    got = _run_world(case, world, K, partition)
    for r in range(world):
        rec, props = got[r][4], got[r][5]
        assert props == [1, 1], props  # one propagation per call, the first included
        if partition == "auto":  # the rule: tiny graphs replicate, no trials
            n, F = case["X"].shape
            assert rec["chosen"] == rule_choice(world, n, len(case["vals"]), F, K) == "replicate"
            assert rec["how"] == "rule" and rec["seconds"] is None
        else:
            assert rec is None


@pytest.mark.parametrize("world,name,chosen", [(4, "norm_n48_F602", "lines"),
                                               (4, "hub1000_F65", "features"),
                                               (2, "norm_n48_F602", "replicate")])
def test_auto_first_call_runs_one_partition(tiny_cases, world, name, chosen):
    """the first call (the one reddit.py:43 times) runs
    exactly one partition's propagation, the rule's, with no trials; the
    minimum-work gate off so the rule picks a split at world >= 3."""
    got = _run_world(tiny_cases[name], world, 2, "auto", env={"SGC_AMD_AUTO_MIN_WORK": "0"},
                     calls=3)
    for r in range(world):
        rec, props = got[r][4], got[r][5]
        assert props == [1, 1, 1], props
        assert rec["chosen"] == chosen and rec["how"] == "rule", rec


@pytest.mark.parametrize("trace", [False, True])
def test_setup_stage_trace(tiny_cases, trace):
    """SGC_AMD_SETUP_TRACE=1 records the first partitioned call's set-up
    stages (the propagator's build, each propagation) by name, for the
    first-call measurements (tests/rank_precompute.py); unset, nothing is
    recorded and the results are the same bits."""
    env = {"SGC_AMD_SETUP_TRACE": "1"} if trace else None
    got = _run_world(tiny_cases["hub1000_F130"], 3, 2, "lines", env=env, calls=2)
    for r in range(3):
        setup = got[r][6]
        if trace:
            assert {"build_lines", "propagate_1", "propagate_2"} <= set(setup), setup
            assert all(v >= 0 for v in setup.values())
        else:
            assert setup == {}


def test_tune_times_on_the_second_call_and_persists(tiny_cases, tmp_path):
    """"tune": the first call runs the rule's partition only; the second times
    every candidate (warm + timed each, plus the winner's result), the third
    runs the winner once; the choice is persisted and a later process's
    "auto" first call takes it (rank 0's file, broadcast) -- still one
    propagation."""
    from sgc_amd.multigpu import AUTO_CANDIDATES
    case = tiny_cases["norm_n48_F602"]
    env = {"SGC_AMD_TUNE_FILE": str(tmp_path / "partitions.json"), "SGC_AMD_AUTO_MIN_WORK": "0"}
    got = _run_world(case, 4, 2, "tune", env=env, calls=3)
    chosen = got[0][4]["chosen"]
    for r in range(4):
        rec, props = got[r][4], got[r][5]
        assert props == [1, 2 * len(AUTO_CANDIDATES) + 1, 1], props
        assert rec["how"] == "timed" and rec["chosen"] == chosen
        assert set(rec["seconds"]) == set(AUTO_CANDIDATES)
    assert (tmp_path / "partitions.json").exists()
    got = _run_world(case, 4, 2, "auto", env=env, calls=2)
    for r in range(4):
        rec, props = got[r][4], got[r][5]
        assert props == [1, 1] and rec["how"] == "persisted" and rec["chosen"] == chosen, rec


def test_single_process_is_untouched(monkeypatch):
    """No torchrun environment, no group: process_group() is None and
    sgc_precompute stays on one device; SGC_AMD_AUTO_DIST=0 also opts out."""
    from sgc_amd import multigpu
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        monkeypatch.delenv(k, raising=False)
    assert multigpu.torchrun_env() is None
    assert multigpu.process_group(torch.device("cpu")) is None
    monkeypatch.setenv("WORLD_SIZE", "2")
    monkeypatch.setenv("RANK", "0")
    monkeypatch.setenv("SGC_AMD_AUTO_DIST", "0")
    assert multigpu.process_group(torch.device("cpu")) is None
    assert multigpu.torchrun_env() == (0, 2, 0, 2)


def test_devices_from_env(monkeypatch):
    from sgc_amd import multigpu
    monkeypatch.delenv("SGC_AMD_DEVICES", raising=False)
    assert multigpu.devices_from_env(0) is None
    monkeypatch.setenv("SGC_AMD_DEVICES", "2,0,1")
    assert multigpu.devices_from_env(1) == [1, 2, 0]  # the caller's device first
    monkeypatch.setenv("SGC_AMD_DEVICES", "0,0,0")    # virtual devices on one GPU
    assert multigpu.devices_from_env(0) == [0, 0, 0]
    monkeypatch.setenv("SGC_AMD_DEVICES", "3")
    assert multigpu.devices_from_env(3) is None


def test_partition_name_checked(monkeypatch):
    from sgc_amd import multigpu
    monkeypatch.setenv("SGC_AMD_PARTITION", "diagonal")
    with pytest.raises(ValueError, match="SGC_AMD_PARTITION"):
        multigpu.partition_name()
    monkeypatch.delenv("SGC_AMD_PARTITION")
    assert multigpu.partition_name() == "auto"
    assert [multigpu.partition_name(w) for w in (2, 3, 4, 8)] == ["auto"] * 4
    assert multigpu.AUTO_CANDIDATES[0] == "replicate"
    # the rule "auto" takes without a persisted choice
    reddit = (232965, 23446803, 602, 2)
    assert [multigpu.rule_choice(w, *reddit) for w in (1, 2, 3, 4, 8)] == \
        ["replicate", "replicate", "lines", "lines", "lines"]
    assert multigpu.rule_choice(8, 232965, 23446803, 200, 2) == "features"  # F < 32 P
    assert multigpu.rule_choice(8, 19717, 108365, 500, 2) == "replicate"    # Pubmed: latency
    monkeypatch.setenv("SGC_AMD_PARTITION", "tune")
    assert multigpu.partition_name() == "tune"
    monkeypatch.setenv("SGC_AMD_PARTITION", "replicate")
    assert multigpu.partition_name(2) == "replicate"
    monkeypatch.setenv("SGC_AMD_PARTITION", "rows")
    assert multigpu.partition_name(8) == "rows"

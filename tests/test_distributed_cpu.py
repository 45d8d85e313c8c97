"""The N>1 path on CPU: world_size 2 over gloo.

The data path itself is per-shard and keyed by the global game id (tested
on the GPU and in test_vec_oracle_game_offset_is_seed_offset); here the
oracle stands in for each rank's device shard so the sharding, the RCCL/
gloo score gather and the Elo replay can be checked without a GPU."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

B, N, EPISODES = 64, 4, 3


def _records(offset, count):
    from oracle import oracle as O

    v = O.VecOracle(count, N, rng_mode=O.RNG_NUMPY_MT, seed=0, game_offset=offset)
    v.reset()
    rew, done, _, _ = v.rollout(10 * EPISODES)
    recs = []
    for e in range(EPISODES):
        scores = rew[10 * e : 10 * e + 10].sum(axis=0)  # [count, N]
        for g in range(count):
            gid = (offset + g) * EPISODES + e
            seats = [(gid + p) % 6 for p in range(N)]  # 6 agents rotate through the seats
            recs.append([gid] + seats + scores[g].tolist())
    return torch.tensor(recs, dtype=torch.int32)


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from rl_6_nimmt.distributed import gather_game_records, reduce_agent_stats, replay_elo, shard

    off, cnt = shard(rank, world, B)
    recs = _records(off, cnt)
    stats = torch.zeros((6, 2), dtype=torch.float64)
    for row in recs.tolist():
        for p in range(N):
            stats[row[1 + p], 0] += 1
            stats[row[1 + p], 1] += row[1 + N + p]
    reduce_agent_stats(stats)
    allrec = gather_game_records(recs)
    elos = replay_elo(allrec, 6, N)
    if rank == 0:
        q.put((stats.numpy(), allrec.numpy(), elos))
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def test_two_rank_gather_equals_single_process():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    stats, allrec, elos = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # single process over the union of the shards
    from rl_6_nimmt.distributed import gather_game_records, replay_elo

    ref = gather_game_records(_records(0, 2 * B))
    assert np.array_equal(allrec, ref.numpy())
    ref_stats = np.zeros((6, 2))
    for row in ref.tolist():
        for p in range(N):
            ref_stats[row[1 + p], 0] += 1
            ref_stats[row[1 + p], 1] += row[1 + N + p]
    assert np.array_equal(stats, ref_stats)
    assert np.allclose(elos, replay_elo(ref, 6, N))


# ---------------------------------------------------------------- batched tournament records
LK, LN, LG = 5, 4, 3


def _league_records(offset, count):
    """this rank's league records, int32 [games, count, 1 + N] for global
    slots offset.., in the device's format: the oracle's restatement of the
    DrunkHamster tournament (oracle.league_records, pinned to the reference's
    seeded tournaments by golden F11 in test_oracle_golden.py; the GPU
    kernel equals it slot for slot, test_gpu_league.py) stands in for the
    rank's device shard"""
    from oracle import oracle as O

    return torch.from_numpy(O.league_records(LK, 2, LN, seed=0, game_offset=offset, slots=count, games=LG))


def _league_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from rl_6_nimmt.distributed import gather_league_records, reduce_agent_stats, shard
    from rl_6_nimmt.league import league_agent_stats, replay_league_elo

    off, cnt = shard(rank, world, B)
    rec = _league_records(off, cnt)
    stats = reduce_agent_stats(league_agent_stats(rec, LK, LN))
    allrec = gather_league_records(rec)
    if rank == 0:
        q.put((stats.numpy(), allrec.numpy(), replay_league_elo(allrec, LK, LN)))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_league_gather_equals_single_process():
    """world_size 2 over gloo: the league's per-agent sums (all_reduce) and the
    gathered records + Elo replay (all_gather, rank order = global slot order)
    equal one process holding every slot."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_league_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    stats, allrec, elos = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    from rl_6_nimmt.league import league_agent_stats, replay_league_elo

    ref = _league_records(0, 2 * B)
    assert np.array_equal(allrec, ref.numpy())
    assert np.allclose(stats, league_agent_stats(ref, LK, LN).numpy())
    assert np.array_equal(elos, replay_league_elo(ref, LK, LN))


# ---------------------------------------------------------------- collective placement (RCCL takes device tensors)
def test_collective_device_follows_the_backend(monkeypatch):
    """RCCL ('nccl': Backend.backend_capability == ['cuda']) takes device
    tensors only, gloo host tensors: the helpers place every collective's
    tensor accordingly (a host tensor on an RCCL group raised "No backend
    type associated with device type cpu" in the round-3 bench)"""
    from rl_6_nimmt import distributed as D

    monkeypatch.setattr(torch.cuda, "current_device", lambda: 3)
    monkeypatch.setattr(dist, "get_backend", lambda group=None: "nccl")
    assert D.collective_device() == torch.device("cuda", 3)
    monkeypatch.setattr(dist, "get_backend", lambda group=None: "gloo")
    assert D.collective_device() == torch.device("cpu")


def _checked_collectives(expected_type, seen):
    """dist.all_reduce / all_gather wrapped to record and check each tensor's device"""
    real_reduce, real_gather = dist.all_reduce, dist.all_gather

    def all_reduce(t, *a, **k):
        seen.append(("all_reduce", t.device.type))
        assert t.device.type == expected_type, t.device
        return real_reduce(t, *a, **k)

    def all_gather(parts, t, *a, **k):
        seen.append(("all_gather", t.device.type))
        assert t.device.type == expected_type and all(p.device.type == expected_type for p in parts)
        return real_gather(parts, t, *a, **k)

    dist.all_reduce, dist.all_gather = all_reduce, all_gather


def _bench_gather_worker(rank, world, port, q):
    """the bench's config-5 score gather (bench_league: host float64 agent
    sums from BatchedTournament.agent_stats, device-side records, the
    max-over-ranks wall) through the helpers, every collective checked to
    receive a tensor on the group's collective device"""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from rl_6_nimmt import distributed as D
    from rl_6_nimmt.league import league_agent_stats

    seen = []
    _checked_collectives(D.collective_device().type, seen)
    off, cnt = D.shard(rank, world, B)
    rec = _league_records(off, cnt)
    stats = D.reduce_agent_stats(league_agent_stats(rec, LK, LN))  # float64, like agent_stats()
    allrec = D.gather_league_records(rec)
    wall = D.max_over_ranks([1.0 + rank, 5.0 - rank])
    if rank == 0:
        q.put((stats.numpy(), allrec.numpy(), wall, seen))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_bench_gather_places_tensors_on_the_collective_device():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bench_gather_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    stats, allrec, wall, seen = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    from rl_6_nimmt.league import league_agent_stats

    ref = _league_records(0, 2 * B)
    assert np.array_equal(allrec, ref.numpy())
    assert np.allclose(stats, league_agent_stats(ref, LK, LN).numpy())
    assert wall == [2.0, 5.0]
    assert {op for op, _ in seen} == {"all_reduce", "all_gather"}


def _gather_to_worker(rank, world, port, q):
    """gather_league_records(rec, dst=0) -- the bench's rank-0
    record gather for the Elo replay (dist.gather through gather_cat_to)"""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from rl_6_nimmt import distributed as D

    off, cnt = D.shard(rank, world, B)
    rec = _league_records(off, cnt)
    got = D.gather_league_records(rec, dst=0)
    every = D.gather_league_records(rec)  # all_gather: the same rows on every rank
    q.put((rank, None if got is None else got.numpy(), every.numpy()))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_gather_to_rank0_equals_all_gather():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gather_to_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict((r, (a, b)) for r, a, b in (q.get(timeout=240) for _ in range(2)))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ref = _league_records(0, 2 * B).numpy()
    assert res[1][0] is None  # dst=0: the other ranks receive nothing
    assert np.array_equal(res[0][0], ref) and np.array_equal(res[0][0], res[0][1])
    assert np.array_equal(res[1][1], ref)


# ---------------------------------------------------------------- bench.py --gpus
def test_bench_gpus_flag_launches_ranks_or_checks_the_launcher(monkeypatch):
    """`bench.py --gpus N`: under a launcher WORLD_SIZE must equal N; without
    one, N > 1 starts torch.distributed.run with N ranks as a child (before
    any GPU call) and returns its exit code"""
    import argparse
    import subprocess
    import sys

    import bench

    ns = lambda g: argparse.Namespace(gpus=g)  # noqa: E731
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    assert bench.resolve_world(ns(None)) == (1, False)
    assert bench.resolve_world(ns(1)) == (1, False)
    assert bench.resolve_world(ns(8)) == (8, True)
    monkeypatch.setenv("WORLD_SIZE", "4")
    assert bench.resolve_world(ns(4)) == (4, False)
    assert bench.resolve_world(ns(None)) == (4, False)
    with pytest.raises(SystemExit):
        bench.resolve_world(ns(2))
    calls = []

    class Done:
        returncode = 7

    monkeypatch.setattr(subprocess, "run", lambda cmd, **k: calls.append(cmd) or Done())
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 8)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "8", "--steps", "5"])
    assert bench.launch_ranks(8) == 7
    cmd = calls[0]
    assert cmd[1:4] == ["-m", "torch.distributed.run", "--nnodes=1"] and "--nproc-per-node=8" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[-4:] == ["--gpus", "8", "--steps", "5"] and cmd[-5].endswith("bench.py")
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 1)
    with pytest.raises(SystemExit):
        bench.launch_ranks(2)

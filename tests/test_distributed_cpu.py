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

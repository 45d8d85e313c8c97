"""Multi-GPU sharding and the tournament score gather.

Games are independent: rank r of W owns global games [r*B, (r+1)*B) and
every random stream is keyed by the global game id, so the union of the
shards is the same set of games as one big handle (no collective on the
data path).  After a block of games:
  * `reduce_agent_stats`: all_reduce(SUM) of per-agent accumulators;
  * `gather_game_records`: all_gather of per-game records (global id, seat
    -> agent, score) so rank 0 can replay the order-dependent Elo updates
    (tournament.py:157-164) in global game-id order;
  * `gather_league_records`: the same for the batched tournament's records
    (league.py), which carry no id column: rank order is global slot order.
    With `dst` the records go to that rank only (dist.gather): the bench's
    Elo replay runs on rank 0 alone; a distributed BatchedTournament keeps
    the all_gather, since every rank ranks the same roster for `evolve`.
Works with any torch.distributed backend (nccl = RCCL on the GPUs, gloo on
CPU): every helper hands the collective a tensor on the device the process
group's backend takes (`collective_device`: RCCL takes device tensors only,
`Backend.backend_capability['nccl'] == ['cuda']`) and returns the result on
the caller's device, so callers may pass host or device tensors alike.
The helpers run the collective whenever a process group is initialised,
world size 1 included (a one-rank RCCL group then exercises the same
device placement the N-rank run needs).
"""
import numpy as np
import torch
import torch.distributed as dist


def shard(rank, world, games_per_rank):
    """(game_offset, num_games) of this rank's shard."""
    return rank * games_per_rank, games_per_rank


def group_active():
    return dist.is_available() and dist.is_initialized()


def world_size():
    return dist.get_world_size() if group_active() else 1


def collective_device(group=None):
    """the device the process group's collectives take tensors on: the
    current GPU for backends that only take device tensors (nccl = RCCL),
    else the host (gloo and the other host-capable backends)"""
    backend = str(dist.get_backend(group))
    caps = dist.Backend.backend_capability.get(backend, ["cpu"])
    if "cpu" in caps:
        return torch.device("cpu")
    return torch.device("cuda", torch.cuda.current_device())


def _on(t, dev):
    return t if t.device == dev else t.to(dev)


def reduce_agent_stats(stats, op=None):
    """stats: float64 tensor [K, F] of per-agent sums (games, score, wins,
    position), reduced in place over the ranks (and returned)."""
    if group_active():
        c = _on(stats.contiguous(), collective_device())
        dist.all_reduce(c, op=dist.ReduceOp.SUM if op is None else op)
        if c.data_ptr() != stats.data_ptr():
            stats.copy_(c.to(stats.device))
    return stats


def all_gather_cat(t, dim=0):
    """every rank's `t` (same shape on every rank) concatenated along `dim`
    in rank order, on t's device"""
    if not group_active():
        return t
    c = _on(t.contiguous(), collective_device())
    parts = [torch.empty_like(c) for _ in range(dist.get_world_size())]
    dist.all_gather(parts, c)
    return torch.cat(parts, dim=dim).to(t.device)


def gather_cat_to(t, dst=0, dim=0):
    """every rank's `t` (same shape on every rank) concatenated along `dim`
    in rank order on rank `dst` (on t's device); None on the other ranks"""
    if not group_active():
        return t
    c = _on(t.contiguous(), collective_device())
    if dist.get_rank() == dst:
        parts = [torch.empty_like(c) for _ in range(dist.get_world_size())]
        dist.gather(c, parts, dst=dst)
        return torch.cat(parts, dim=dim).to(t.device)
    dist.gather(c, None, dst=dst)
    return None


def backend_label():
    """the collective library the process group runs on, for result lines"""
    if not group_active():
        return "single process (no collective)"
    b = str(dist.get_backend())
    return "RCCL" if b == "nccl" else b


def gather_game_records(records):
    """records: int32 tensor [G, 1 + 2*N] rows (global game id, seat agent ids, seat scores),
    same G on every rank.  Returns all ranks' rows sorted by global game id."""
    records = all_gather_cat(records, dim=0)
    order = torch.argsort(records[:, 0].to(torch.int64), stable=True)
    return records[order]


def gather_league_records(records, dst=None):
    """Batched-tournament records of this rank, int32 [games, slots, 1 + N]
    (rank r owns global slots [r*slots, (r+1)*slots)), gathered (RCCL on the
    GPUs) into [games, world*slots, 1 + N]: round major, then global slot id
    -- the canonical order of the Elo replay (league.replay_league_elo).
    dst=None: on every rank (all_gather); dst=r: on rank r only, None on the
    others (dist.gather -- the Elo replay needs them on one rank)."""
    if dst is None:
        return all_gather_cat(records, dim=1)
    return gather_cat_to(records, dst=dst, dim=1)


def max_over_ranks(values, device=None):
    """elementwise max of a list of floats over the ranks (wall times)"""
    t = torch.tensor(list(values), dtype=torch.float64, device=device)
    if group_active():
        reduce_agent_stats(t, op=dist.ReduceOp.MAX)
    return [float(x) for x in t.tolist()]


def replay_elo(records, num_agents, num_players, elo_initial=1600.0, elo_k=32.0):
    """Sequential multiplayer Elo over gathered records (host, global game order)."""
    from .elo import EloPlayer, calc_elo
    from .tournament import Tournament

    elos = np.full(num_agents, float(elo_initial))
    rec = records.cpu().numpy()
    for row in rec:
        seats = row[1 : 1 + num_players]
        scores = row[1 + num_players : 1 + 2 * num_players]
        places = Tournament._compute_absolute_positions(scores)
        new = calc_elo([EloPlayer(pl, elos[a]) for pl, a in zip(places, seats)], elo_k)
        for a, e in zip(seats, new):
            elos[a] = e
    return elos

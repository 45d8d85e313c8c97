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
Works with any torch.distributed backend (nccl = RCCL on the GPUs, gloo on CPU).
"""
import numpy as np
import torch
import torch.distributed as dist


def shard(rank, world, games_per_rank):
    """(game_offset, num_games) of this rank's shard."""
    return rank * games_per_rank, games_per_rank


def reduce_agent_stats(stats):
    """stats: float64 tensor [K, F] of per-agent sums (games, score, wins, position)."""
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(stats, op=dist.ReduceOp.SUM)
    return stats


def gather_game_records(records):
    """records: int32 tensor [G, 1 + 2*N] rows (global game id, seat agent ids, seat scores),
    same G on every rank.  Returns all ranks' rows sorted by global game id."""
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        parts = [torch.empty_like(records) for _ in range(dist.get_world_size())]
        dist.all_gather(parts, records)
        records = torch.cat(parts, dim=0)
    order = torch.argsort(records[:, 0].to(torch.int64), stable=True)
    return records[order]


def gather_league_records(records):
    """Batched-tournament records of this rank, int32 [games, slots, 1 + N]
    (rank r owns global slots [r*slots, (r+1)*slots)), all_gather'ed (RCCL on
    the GPUs) into [games, world*slots, 1 + N]: round major, then global slot
    id -- the canonical order of the Elo replay (league.replay_league_elo)."""
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        parts = [torch.empty_like(records) for _ in range(dist.get_world_size())]
        dist.all_gather(parts, records.contiguous())
        records = torch.cat(parts, dim=1)
    return records


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

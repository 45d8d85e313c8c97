"""GPU parity of the batched tournament (league.py, BASELINE config 5).

* slot g of a tournament handle replays the reference's
  `np.random.seed(seed + g); Tournament(min, max) over K DrunkHamster agents;
  play_game() x games` -- seat draws, results -- bit for bit (golden F11,
  tests/golden/tournament_games.json, recorded from the reference itself);
* at the bench's size (65 536 slots): records independent of the sharding
  (two half-size handles == one handle), per-game invariants of the scoring
  (relative positions of a game sum to k/2, one winner per game, Elo sum
  conserved), agent ids distinct per game.
"""
import json
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN

pytestmark = pytest.mark.gpu


def load(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def _league(B, K, lo, hi, seed, game_offset=0, rng="numpy"):
    from rl_6_nimmt.league import BatchedTournament

    t = BatchedTournament(B, lo, hi, seed=seed, game_offset=game_offset, rng=rng)
    for i in range(K):
        t.add_player(f"a{i}")
    return t


def test_league_slots_replay_reference_tournaments():
    from rl_6_nimmt.league import decode_seats

    groups = {}
    for r in load("tournament_games.json")["league"]:
        groups.setdefault((r["num_agents"], r["min_players"], r["max_players"]), []).append(r)
    assert len(groups) == 3
    for (K, lo, hi), recs in groups.items():
        base = recs[0]["seed"]
        assert [r["seed"] for r in recs] == list(range(base, base + len(recs)))
        games = len(recs[0]["results"])
        t = _league(len(recs), K, lo, hi, seed=base)
        rec = t.play_games(games).cpu()
        k, ids = decode_seats(rec[..., 0], hi)
        for j, r in enumerate(recs):
            for e in range(games):
                seats, res = r["seats"][e], r["results"][e]
                assert int(k[e, j]) == len(seats), (K, lo, hi, j, e)
                assert ids[e, j, : len(seats)].tolist() == seats, (K, lo, hi, j, e)
                assert rec[e, j, 1: 1 + len(seats)].tolist() == res, (K, lo, hi, j, e)
                assert not rec[e, j, 1 + len(seats):].any()
        assert t.env.pipe_errors() == 0
        t.close()


@pytest.mark.parametrize("rng", ["numpy", "philox"])
def test_league_full_size_sharding_and_scoring_invariants(rng):
    from rl_6_nimmt.league import decode_seats, relative_positions, winners

    B, K, lo, hi, G = 65536, 5, 2, 4, 3
    t = _league(B, K, lo, hi, seed=7, rng=rng)
    rec = t.play_games(G)
    t2 = _league(B // 2, K, lo, hi, seed=7, game_offset=B // 2, rng=rng)
    rec2 = t2.play_games(G)
    assert torch.equal(rec[:, B // 2:], rec2)
    k, ids = decode_seats(rec[..., 0], hi)
    assert int(k.min()) >= lo and int(k.max()) <= hi
    counts = torch.bincount(k.reshape(-1), minlength=hi + 1)[lo:].cpu().numpy()
    assert counts.min() > 0.3 * counts.max()  # every player count occurs (uniform choice)
    valid = ids >= 0
    assert int(ids.max()) < K
    s = torch.sort(torch.where(valid, ids, 100 + torch.arange(hi, device=ids.device)), dim=-1).values
    assert not (s[..., 1:] == s[..., :-1]).any()  # distinct agents per game (replace=False)
    res = rec[..., 1:]
    pen = -res.sum(dim=-1)
    assert int(res.max()) <= 0 and int(pen.max()) <= 171
    assert not res[~valid].any()
    rel = relative_positions(res, k)
    assert torch.allclose(rel.sum(dim=-1), k.double() / 2)
    w = winners(res, k)
    assert bool((w < k).all())
    stats = t.agent_stats()
    assert int(stats[:, 0].sum()) == int(k.sum())
    assert int(stats[:, 3].sum()) == G * B
    elos = t.replay_elo()
    assert abs(elos.sum() - K * 1600.0) < 1e-6 * K * 1600.0  # pairwise Elo exchanges conserve the sum
    if rng == "numpy":
        assert t.env.pipe_errors() == 0 and t2.env.pipe_errors() == 0
    t.close()
    t2.close()


def _mixed(B, specs, lo, hi, seed, game_offset=0, fused=False, train=False):
    """a tournament over (name, agent) specs"""
    from rl_6_nimmt.league import BatchedTournament

    t = BatchedTournament(B, lo, hi, seed=seed, game_offset=game_offset, fused=fused, train=train)
    for name, agent in specs:
        t.add_player(name, agent)
    return t


def test_dropin_leagues_replay_reference_tournaments_batched():
    """golden F11 "dropin" leagues (DrunkHamster + MCSAgent seats, seeded
    reference Tournament.play_game x games): the batched tournament's slot 0
    (sn_reset seat draw + deal, 10 sn_league_step launches per game, the MCS
    seats' reference-exact search on the slot's stream) replays every seat
    draw, result, relative position and winner, and the tallies"""
    from rl_6_nimmt.agents import DrunkHamster, MCSAgent
    from rl_6_nimmt.league import decode_seats, relative_positions, winners

    for lg in load("tournament_games.json")["dropin"]:
        specs = [(n, MCSAgent(mc_max=lg["mc_max"], mc_per_card=lg["mc_per_card"]) if c == "M" else DrunkHamster())
                 for n, c in zip(lg["agents"], lg["kinds"])]
        G, hi = len(lg["games"]), lg["max_players"]
        t = _mixed(3, specs, lg["min_players"], hi, seed=lg["seed"])
        rec = t.play_games(G).cpu()
        assert t.mode == "step"
        k, ids = decode_seats(rec[..., 0], hi)
        res = rec[..., 1:]
        rel, win = relative_positions(res, k), winners(res, k)
        for e, g in enumerate(lg["games"]):
            kk = len(g["names"])
            assert int(k[e, 0]) == kk, (lg["kinds"], e)
            assert [lg["agents"][i] for i in ids[e, 0, :kk].tolist()] == g["names"], (lg["kinds"], e)
            assert res[e, 0, :kk].tolist() == g["results"], (lg["kinds"], e)
            assert np.allclose(rel[e, 0, :kk].numpy(), g["relative"]), (lg["kinds"], e)
            assert g["names"][int(win[e, 0])] == g["winner"]
        # tallies of the slot-0 tournament (tournament.py:147-152)
        st = t.agent_stats(rec[:, :1])
        for i, n in enumerate(lg["agents"]):
            ref = lg["tallies"][n]
            assert int(st[i, 0]) == ref["played_games"], n
            assert int(st[i, 1]) == sum(ref["scores"]), n
            assert abs(float(st[i, 2]) - sum(ref["positions"])) < 1e-6, n  # the reference's positions are float32
            assert int(st[i, 3]) == int(sum(ref["wins"])), n
        t.close()


def test_league_step_mode_equals_fused_rollout():
    """an all-DrunkHamster league played round by round (sn_reset +
    sn_league_step) draws the same words in the same order as the fused
    sn_league_rollout: identical records"""
    B, K, lo, hi, G = 4096, 5, 2, 4, 3
    t1 = _league(B, K, lo, hi, seed=11)
    r1 = t1.play_games(G)
    from rl_6_nimmt.agents import DrunkHamster

    t2 = _mixed(B, [(f"a{i}", DrunkHamster()) for i in range(K)], lo, hi, seed=11, fused=False)
    r2 = t2.play_games(1)
    r2 = torch.cat((r2, t2.play_games(G - 1)), dim=0)
    assert t1.mode == "fused" and t2.mode == "step"
    assert torch.equal(r1, r2)
    assert np.allclose(t1.replay_elo(), t2.replay_elo())
    t1.close()
    t2.close()


def _run_py_pool(mc_max=200):
    """run.py:24-27's league plus the random agent of its notebook stage"""
    from rl_6_nimmt.agents import BatchedACERAgent, DrunkHamster, MCSAgent, PUCTAgent, PUCTCustomedAgent

    torch.manual_seed(0)
    return [("ACER", BatchedACERAgent(minibatch=10)), ("MCS", MCSAgent(mc_max=mc_max)),
            ("Alpha0.5", PUCTAgent(mc_max=mc_max)), ("Alpha0.5_customed", PUCTCustomedAgent(mc_max=mc_max)),
            ("Random", DrunkHamster())]


def test_mixed_league_with_net_agents_plays_and_trains():
    """a run.py-seated league (ACER, MCS, Alpha0.5, Alpha0.5_customed at
    mc_max=200, plus Random) on 256 slots, training on: every move legal
    (sn_league_step checks the engines' cards), records well formed, tallies
    and Elo consistent, and every net agent's weights move"""
    from rl_6_nimmt.league import decode_seats, relative_positions

    specs = _run_py_pool(mc_max=20)
    before = {n: [p.detach().clone() for p in a.parameters()] for n, a in specs if n not in ("MCS", "Random")}
    for n, a in specs:
        if n not in ("MCS", "Random"):  # run.py:29-33 (its try/except skips the parameter-free agents)
            a.train()
    B, lo, hi, G = 256, 2, 4, 2
    t = _mixed(B, specs, lo, hi, seed=3, train=True)
    rec = t.play_games(G)
    k, ids = decode_seats(rec[..., 0], hi)
    assert int(k.min()) >= lo and int(k.max()) <= hi and int(ids.max()) < len(specs)
    valid = ids >= 0
    res = rec[..., 1:]
    assert int(res.max()) <= 0 and int((-res.sum(-1)).max()) <= 171 and not res[~valid].any()
    assert torch.allclose(relative_positions(res, k).sum(-1), k.double() / 2)
    st = t.agent_stats()
    assert int(st[:, 0].sum()) == int(k.sum()) and int(st[:, 3].sum()) == G * B
    assert all(st[i, 0] > 0 for i in range(len(specs)))
    assert abs(t.replay_elo().sum() - len(specs) * 1600.0) < 1e-6
    for n, ps in before.items():
        now = list(t.agents[n].parameters())
        assert any(not torch.equal(a.cpu(), b.cpu()) for a, b in zip(now, ps)), n
    t.close()


def test_mixed_league_evolve_reseats_the_new_roster():
    """Tournament.evolve between rounds (tournament.py:78-130): clones join,
    pruned agents leave, and the next round's seats come from the new active
    list (seat ids index it)"""
    from rl_6_nimmt.agents import DrunkHamster, MCSAgent
    from rl_6_nimmt.league import decode_seats

    specs = [("R0", DrunkHamster()), ("M", MCSAgent(mc_max=20)), ("R1", DrunkHamster()), ("R2", DrunkHamster())]
    t = _mixed(512, specs, 2, 4, seed=5)
    t.play_games(1)
    t.evolve(copies=(2,), max_players=4, max_per_descendant=2, metric="tournament_scores")
    act = t.active_agents()
    assert len(act) == 4 and len(t.names) == 5  # best x2, two more x1, the worst deactivated (max_players)
    rec = t.play_games(1)
    k, ids = decode_seats(rec[..., 0], 4)
    assert int(ids.max()) == len(act) - 1  # 512 slots: every active agent is seated somewhere
    st = t.agent_stats()
    assert int(st[:, 0].sum()) >= int(k.sum())
    t.close()


def test_league_records_equal_oracle_shards():
    """the device's records of a rank's shard (game_offset) equal the
    oracle's tournament restatement -- what the 2-rank gloo test
    (test_distributed_cpu.py) gathers in place of device records"""
    from oracle import oracle as O

    for off in (0, 96):
        t = _league(96, 5, 2, 4, seed=0, game_offset=off)
        rec = t.play_games(3).cpu().numpy()
        assert np.array_equal(rec, O.league_records(5, 2, 4, seed=0, game_offset=off, slots=96, games=3))
        t.close()


def _rank_league(rank, world, port, q, B, G):
    """one rank of the distributed league on cuda:0: its shard of device
    slots, the per-agent all_reduce and the record all_gather (gloo here --
    two ranks cannot share one GPU under RCCL; bench.py uses nccl = RCCL)"""
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from rl_6_nimmt.distributed import gather_league_records, reduce_agent_stats, shard

    off, cnt = shard(rank, world, B)
    t = _league(cnt, 5, 2, 4, seed=3, game_offset=off)
    t.play_games(G)
    stats = reduce_agent_stats(t.agent_stats().cpu())
    allrec = gather_league_records(t.all_records().cpu())
    errs = t.env.pipe_errors()
    t.close()
    if rank == 0:
        q.put((stats.numpy(), allrec.numpy(), errs))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_device_league_gather_equals_one_handle():
    """world_size 2 with DEVICE records: each rank plays its shard of slots
    on the GPU; the gathered records and the reduced per-agent sums equal one
    handle holding every slot (the CPU gloo test gathers oracle records)."""
    import socket

    import torch.multiprocessing as mp

    from rl_6_nimmt.league import replay_league_elo

    B, G = 512, 3
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_rank_league, args=(r, 2, port, q, B, G)) for r in range(2)]
    for p in procs:
        p.start()
    stats, allrec, errs = q.get(timeout=180)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    t = _league(2 * B, 5, 2, 4, seed=3)
    t.play_games(G)
    ref = t.all_records().cpu().numpy()
    assert errs == 0 and t.env.pipe_errors() == 0
    assert allrec.shape == ref.shape and np.array_equal(allrec, ref)
    assert np.allclose(stats, t.agent_stats().cpu().numpy())
    assert np.allclose(replay_league_elo(torch.from_numpy(allrec), 5, 4), t.replay_elo(), rtol=0, atol=1e-9)
    t.close()


def _rccl_one_rank(port, q):
    """a one-rank RCCL (backend 'nccl') group: the bench's config-5 legs run
    their score gathers through it -- the collectives then take exactly the
    device placement an N-rank RCCL run needs"""
    import torch.distributed as dist

    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, init_method=f"tcp://127.0.0.1:{port}",
                           device_id=torch.device("cuda", 0))
    import bench
    from rl_6_nimmt import distributed as D

    assert D.collective_device().type == "cuda"
    host = D.reduce_agent_stats(torch.ones((3, 4), dtype=torch.float64))  # a host tensor through RCCL
    assert host.device.type == "cpu" and bool((host == 1).all())
    league = bench.bench_league(1, 0, 2048, 2)
    mixed = bench.bench_league_mixed(1, 0, 256, mc_max=10)
    wall = D.max_over_ranks([1.5, 2.5], device=torch.device("cuda", 0))
    dist.destroy_process_group()
    q.put((league["agents"], mixed["agents"], wall))


def test_rccl_group_runs_the_bench_score_gathers():
    """round 3 handed RCCL a host tensor (BatchedTournament.agent_stats) and
    the N>1 bench died at its config-5 leg; every collective of the bench's
    league legs now goes through a one-rank RCCL group on the GPU"""
    import socket

    import torch.multiprocessing as mp

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_rccl_one_rank, args=(port, q))
    p.start()
    league, mixed, wall = q.get(timeout=240)
    p.join(timeout=60)
    assert p.exitcode == 0
    assert sum(a["games"] for a in league.values()) > 0 and sum(a["games"] for a in mixed.values()) > 0
    assert wall == [1.5, 2.5]


def _f13():
    return load("evolve_games.json")["cases"]


def _roster_names(roster):
    return [r["name"] for r in roster]


@pytest.mark.parametrize("ci", range(5))
def test_batched_league_with_evolve_replays_reference(ci):
    """golden F13 end to end on the GPU: a one-slot tournament handle
    (np.random.seed(seed) stream: seat draws over the CURRENT active list,
    deals and DrunkHamster moves in-kernel) plays every block's games, evolve
    runs between blocks -- every game's seats and results and the roster
    after every evolve equal the reference tournament's
    (tournament.py:54-177)"""
    from rl_6_nimmt.league import decode_seats

    case = _f13()[ci]
    hi = case["max_players"]
    from rl_6_nimmt.agents import DrunkHamster

    t = _mixed(1, [(f"a{i}", DrunkHamster())
                   for i in range(case["num_agents"])], case["min_players"], hi, seed=case["seed"])
    for block in case["blocks"]:
        active = t.active_agents()
        rec = t.play_games(len(block["games"])).cpu()
        k, ids = decode_seats(rec[..., 0], hi)
        for e, g in enumerate(block["games"]):
            kk = len(g["names"])
            assert int(k[e, 0]) == kk
            assert [active[i] for i in ids[e, 0, :kk].tolist()] == g["names"], (ci, e)
            assert rec[e, 0, 1: 1 + kk].tolist() == g["results"], (ci, e)
        if "evolve" in block:
            ev = dict(block["evolve"])
            ev["copies"] = tuple(ev["copies"])
            t.evolve(**ev)
            assert t.names == _roster_names(block["after"])
            assert [t.active[n] for n in t.names] == [r["active"] for r in block["after"]]
            st = t.agent_stats().numpy()
            assert st[:, 0].tolist() == [r["played_games"] for r in block["after"]]
            assert t.elos.tolist() == [r["elo"] for r in block["after"]]
    assert t.env.pipe_errors() == 0
    t.close()


def test_dropin_tournament_with_evolve_replays_reference():
    """the drop-in Tournament (host league over the one-game device env) on
    golden F13: np.random.seed(seed), play_game x games, evolve between blocks"""
    from rl_6_nimmt import Tournament
    from rl_6_nimmt.agents import DrunkHamster

    for case in _f13()[:3]:
        np.random.seed(case["seed"])
        t = Tournament(case["min_players"], case["max_players"])
        for i in range(case["num_agents"]):
            t.add_player(f"a{i}", DrunkHamster())
        for block in case["blocks"]:
            for g in block["games"]:
                t.play_game()
            if "evolve" in block:
                ev = dict(block["evolve"])
                ev["copies"] = tuple(ev["copies"])
                for r in block["before"]:
                    assert [int(x) for x in t.tournament_scores[r["name"]]] == r["scores"]
                t.evolve(**ev)
                assert list(t.agents.keys()) == _roster_names(block["after"])
                assert [t.elos[n][-1] for n in t.agents] == [r["elo"] for r in block["after"]]


def test_mixed_league_every_slot_equals_oracle():
    """DrunkHamster + MCSAgent league (reference-exact MCS on each slot's
    numpy stream, sn_league_step) at 512 slots x 3 games: EVERY slot's
    records equal the oracle's restatement (oracle.league_mixed_records,
    itself pinned to golden F11's seeded reference tournaments)"""
    from oracle import oracle as O
    from rl_6_nimmt.agents import DrunkHamster, MCSAgent

    kinds, B, G = "RMRMR", 512, 3
    specs = [(f"{c}{i}", MCSAgent(mc_max=100) if c == "M" else DrunkHamster()) for i, c in enumerate(kinds)]
    t = _mixed(B, specs, 2, 4, seed=77)
    rec = t.play_games(G).cpu().numpy()
    ref, q6 = O.league_mixed_records(kinds, 2, 4, mc_per_card=10, mc_max=100, seed=77, slots=B, games=G)
    assert t.mode == "step"
    bad = np.nonzero((rec != ref).any(axis=(0, 2)))[0]
    assert bad.size == 0, f"slots differing from the oracle: {bad[:10].tolist()}"
    assert (t.q6_slot_rounds > 0) == (int(q6.sum()) > 0)
    assert t.env.pipe_errors() == 0
    t.close()


def test_mixed_league_full_size_sharding_invariance():
    """65 536-slot DrunkHamster + MCSAgent league: two half-size handles
    (game_offset) give exactly the records of one full handle, and a sample
    of slots equals the oracle"""
    from oracle import oracle as O
    from rl_6_nimmt.agents import DrunkHamster, MCSAgent

    kinds, B = "RMRRM", 65536

    def specs():
        return [(f"{c}{i}", MCSAgent(mc_max=100) if c == "M" else DrunkHamster()) for i, c in enumerate(kinds)]

    t = _mixed(B, specs(), 2, 4, seed=9)
    rec = t.play_games(1)
    h = [_mixed(B // 2, specs(), 2, 4, seed=9, game_offset=o) for o in (0, B // 2)]
    halves = torch.cat([x.play_games(1) for x in h], dim=1)
    assert torch.equal(rec, halves)
    ref, _ = O.league_mixed_records(kinds, 2, 4, seed=9, game_offset=B - 64, slots=64, games=1)
    assert np.array_equal(rec[:, B - 64:].cpu().numpy(), ref)
    for x in [t] + h:
        assert x.env.pipe_errors() == 0
        x.close()


def test_league_seats_a_reinforce_agent_and_trains_it():
    """BatchedReinforceAgent (agents/policy.py:109-201) takes a seat in the
    batched tournament: its engine samples on its seats' decision list, every
    move is legal (sn_league_step checks), and one REINFORCE step per round
    moves its weights"""
    from rl_6_nimmt.agents import BatchedReinforceAgent, DrunkHamster, MCSAgent

    torch.manual_seed(1)
    rf = BatchedReinforceAgent()
    rf.train()
    before = [p.detach().clone() for p in rf.parameters()]
    specs = [("R0", DrunkHamster()), ("REINFORCE", rf), ("M", MCSAgent(mc_max=20)), ("R1", DrunkHamster())]
    t = _mixed(256, specs, 2, 4, seed=12, train=True)
    rec = t.play_games(2)
    from rl_6_nimmt.league import decode_seats

    k, ids = decode_seats(rec[..., 0], 4)
    assert int((ids == 1).sum()) > 0  # the REINFORCE agent was seated
    st = t.agent_stats()
    assert int(st[:, 0].sum()) == int(k.sum()) and int(st[1, 0]) > 0
    assert any(not torch.equal(a.detach().cpu(), b.cpu()) for a, b in zip(t.agents["REINFORCE"].parameters(), before))
    assert t.env.pipe_errors() == 0
    t.close()


def test_batched_baseline_evaluations():
    """Tournament(baseline_agents=...) (tournament.py:147-155,182-195): every
    time an agent's game count reaches a multiple of baseline_condition it
    gets one evaluation -- GameSession(agent, *baseline_agents) x
    baseline_num_games, per-seat mean scores, the agent's relative position
    and win flag -- here batched on a handle of its own"""
    from rl_6_nimmt.agents import DrunkHamster, MCSAgent

    from rl_6_nimmt.league import BatchedTournament

    base = [DrunkHamster(), DrunkHamster()]
    t = BatchedTournament(16, 2, 3, seed=4, fused=False, baseline_agents=base, baseline_num_games=2, baseline_condition=3)
    for i in range(3):
        t.add_player(f"R{i}", DrunkHamster())
    t.add_player("M", MCSAgent(mc_max=20))
    t.play_games(2)
    st = t.agent_stats().numpy()
    for i, n in enumerate(t.names):
        k = int(st[i, 0]) // 3
        assert len(t.baseline_scores[n]) == k and len(t.baseline_positions[n]) == k and len(t.baseline_wins[n]) == k, n
        assert all(-171 <= v <= 0 for v in t.baseline_scores[n])
        assert all(0.0 <= v <= 1.0 for v in t.baseline_positions[n])
        assert set(t.baseline_wins[n]) <= {0.0, 1.0}
        assert t.agents[n].__name__ == n
    assert sum(len(v) for v in t.baseline_scores.values()) > 0
    t.close()


def _dist_tournament(B, seed, game_offset, distributed, condition=128):
    from rl_6_nimmt.agents import DrunkHamster, MCSAgent
    from rl_6_nimmt.league import BatchedTournament

    t = BatchedTournament(B, 2, 4, seed=seed, game_offset=game_offset, rng="numpy", fused=False,
                          distributed=distributed, baseline_agents=[DrunkHamster(), DrunkHamster()],
                          baseline_condition=condition)
    for i in range(4):
        t.add_player(f"a{i}")
    t.add_player("mcs", MCSAgent(mc_max=10))
    t.play_games(2)
    t.evolve(copies=(2,), max_players=5)
    t.play_games(1)
    w = t.winner()
    out = {"names": list(t.names), "active": dict(t.active), "stats": t.agent_stats().numpy(),
           "elos": t.replay_elo(), "total": t.total_games, "table": str(t),
           "positions": {n: np.concatenate(p) if p else np.zeros(0) for n, p in t.positions.items()},
           "baseline": {n: list(v) for n, v in t.baseline_scores.items()},
           "winner": getattr(w, "__name__", None), "errs": t.env.pipe_errors()}
    t.close()
    return out


def _rank_dist_tournament(rank, world, port, q, B):
    """one rank of a distributed=True tournament on cuda:0 (gloo: two ranks
    cannot share one GPU under RCCL): play, evolve, play, then every
    accessor -- each a collective on every rank"""
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    out = _dist_tournament(B, 5, rank * B, True)
    got = [None] * world
    dist.all_gather_object(got, out)
    if rank == 0:
        q.put(got)
    dist.barrier()
    dist.destroy_process_group()


def test_distributed_tournament_keeps_one_roster_on_every_rank():
    """BatchedTournament(distributed=True) on 2 ranks -- play,
    evolve, play -- leaves the SAME roster, tallies, Elo, positions, baseline
    evaluations, winner and table on both ranks, equal to one process holding
    every slot; total_games counts the whole world"""
    import socket

    import torch.multiprocessing as mp

    B = 256
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_rank_dist_tournament, args=(r, 2, port, q, B)) for r in range(2)]
    for p in procs:
        p.start()
    got = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ref = _dist_tournament(2 * B, 5, 0, False)
    for r in got:
        assert r["errs"] == 0
        assert r["names"] == ref["names"] and r["active"] == ref["active"]
        assert np.array_equal(r["stats"], ref["stats"])
        assert np.allclose(r["elos"], ref["elos"], rtol=0, atol=1e-9)
        assert r["total"] == ref["total"] == 3 * 2 * B
        assert r["table"] == ref["table"]
        assert r["winner"] == ref["winner"]
        assert r["baseline"] == ref["baseline"] and any(len(v) for v in ref["baseline"].values())
        for n in ref["positions"]:
            assert np.array_equal(r["positions"][n], ref["positions"][n])


@pytest.mark.parametrize("k", [1, 3, "games"])
def test_updates_per_round_takes_k_adam_steps(k):
    """BatchedTournament(updates_per_round=k): each trained PUCT /
    PUCTCustomed / REINFORCE agent takes k Adam steps per round (k chunks of
    its games); "games" takes one per game it played -- the reference's count
    (learn() at every episode end, play.py:52-67, mcts.py:230-261)"""
    from rl_6_nimmt.agents import BatchedReinforceAgent, PUCTAgent, PUCTCustomedAgent
    from rl_6_nimmt.league import BatchedTournament, decode_seats

    torch.manual_seed(0)
    t = BatchedTournament(48, 2, 4, seed=1, rng="numpy", fused=False, train=True, updates_per_round=k)
    nets = {"p": PUCTAgent(mc_max=6), "c": PUCTCustomedAgent(mc_max=6), "r": BatchedReinforceAgent()}
    for n, a in nets.items():
        a.train()
        t.add_player(n, a)
    t.add_player("x0")
    before = {n: [q.detach().clone() for q in a.parameters()] for n, a in nets.items()}
    rec = t.play_games(1)
    kk, ids = decode_seats(rec[0, :, 0], 4)
    act = t.active_agents()
    for n in nets:
        j = act.index(n)
        games = int(((ids == j) & (torch.arange(4, device=ids.device)[None, :] < kk[:, None])).any(dim=1).sum())
        want = games if k == "games" else min(k, games)
        assert games > 3 and t.optimizer_steps.get(n, 0) == want, (n, games, t.optimizer_steps)
        assert any(not torch.equal(a.cpu(), b.detach().cpu()) for a, b in zip(before[n], nets[n].parameters()))
    t.close()


def test_clone_inherits_the_acer_replay_and_plays():
    """the reference's copy_player round-trips the agent
    through torch.save, so a clone carries its parent's history
    (tournament.py:54-60); the clone's batched ACER engine starts from the
    parent's device replay.  copy_player / remove_player take effect from
    the next game (the handle is reconfigured lazily): the clone is seated."""
    from rl_6_nimmt.agents import BatchedACERAgent
    from rl_6_nimmt.league import BatchedTournament, decode_seats

    torch.manual_seed(0)
    t = BatchedTournament(256, 2, 4, seed=3, rng="numpy", fused=False, train=True)
    a = BatchedACERAgent(minibatch=2)
    a.train()
    t.add_player("acer", a)
    for i in range(3):
        t.add_player(f"r{i}")
    t.play_games(2)
    src = t.engines["acer"]
    assert src.episodes > 0
    t.copy_player("acer", "acer_c")
    t.remove_player("r0")
    t._configure()  # what the next game does first
    dst = t.engines["acer_c"]
    n = min(src.episodes, src.capacity, dst.capacity)
    assert n > 0 and dst.episodes == n
    for k in range(n):
        a_, b_ = (src.episodes - n + k) % src.capacity, k % dst.capacity
        assert torch.equal(dst.rep_rows[b_], src.rep_rows[a_]) and torch.equal(dst.rep_logp[b_], src.rep_logp[a_])
        assert torch.equal(dst.rep_act[b_], src.rep_act[a_]) and torch.equal(dst.rep_rew[b_], src.rep_rew[a_])
    rec = t.play_games(1)
    kk, ids = decode_seats(rec[0, :, 0], 4)
    seated = (ids == t.active_agents().index("acer_c")) & (torch.arange(4, device=ids.device)[None, :] < kk[:, None])
    assert bool(seated.any()) and "r0" not in t.active_agents()
    t.close()

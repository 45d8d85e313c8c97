#!/usr/bin/env python3
"""F14 fixture: seeded reference PUCT search statistics (test infrastructure).

Runs ONLY in the build container: imports the reference from /root/reference
(tools/gen_fixtures.import_reference, with its stand-ins for the absent gym /
numba / multi_elo) and records, per game g of
    np.random.seed(g); torch.manual_seed(10_000 + g)
    GameSession(PUCTAgent(mc_max=20) [F8 weights, eval], DrunkHamster x 3).play_game()
the initial deal, every seat's result, and seat 0's first decision (n = 10):
its legal cards, the PUCT visit count of each and the chosen card
(agents/mcts.py:191-323, play.py:23-75).  The F8 weights are
torch.manual_seed(0); PUCTAgent()'s (checked against puct_policy.npz).

One deviation, stated in the fixture: _choose_action_from_outcomes'
debug f-string (mcts.py:165-170) indexes log_probs[action][0] for EVERY
legal move, so the reference raises IndexError whenever a move got no
playout (quirk Q6) -- here that method is replaced by its decision logic
without the debug lines (same best move, same info), so such games finish
as the batched engine finishes them.  Usage:
    PYTHONDONTWRITEBYTECODE=1 python tools/gen_puct_stats.py [games] [workers]
    SECHS_F14_MC_MAX=100 ... -> F14b, tests/golden/puct_search_mc100.json
"""
import json
import multiprocessing as mp
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
MC_MAX = int(os.environ.get("SECHS_F14_MC_MAX", "20"))
# F14 (mc_max 20, first decision) keeps its file; F14b (mc_max 100, the reference's default budget,
# mcts.py:25) records seat 0's decisions at n = 10, 6 and 3 into its own.
OUT = os.path.join(ROOT, "tests", "golden", "puct_search.json" if MC_MAX == 20 else f"puct_search_mc{MC_MAX}.json")
DEC_N = (10, 6, 3)


def _worker(args):
    lo, hi = args
    import gen_fixtures

    gen_fixtures.import_reference()
    import torch

    torch.set_num_threads(1)  # one core per worker process

    from rl_6_nimmt.agents import DrunkHamster, PUCTAgent
    from rl_6_nimmt.agents.mcts import BaseMCAgent
    from rl_6_nimmt.play import GameSession

    first = {}

    def choose(self, outcomes, log_probs):
        # mcts.py:159-163's decision (first maximum of the outcome means) without the debug lines
        best_action, best_mean = list(outcomes.keys())[0], -float("inf")
        for action, outcome in outcomes.items():
            if np.mean(outcome) > best_mean:
                best_action, best_mean = action, np.mean(outcome)
        n = len(outcomes)
        if n in DEC_N and getattr(self, "_seat0", False) and str(n) not in first.setdefault("dec", {}):
            first["dec"][str(n)] = {"legal": [int(a) for a in outcomes], "visits": [len(o) for o in outcomes.values()],
                                    "chosen": int(best_action)}
            if n == 10:
                first["legal"], first["visits"], first["chosen"] = (first["dec"]["10"][k] for k in ("legal", "visits", "chosen"))
        return best_action, {"log_prob": log_probs[best_action][0]}

    BaseMCAgent._choose_action_from_outcomes = choose
    torch.manual_seed(0)
    puct = PUCTAgent(mc_max=MC_MAX)
    z = np.load(os.path.join(ROOT, "tests", "golden", "puct_policy.npz"))
    for k, v in puct.actor.state_dict().items():
        assert np.array_equal(v.numpy(), z[k]), k  # the F8 weights
    puct.eval()
    puct._seat0 = True
    recs = []
    np.seterr(all="ignore")
    import warnings

    warnings.simplefilter("ignore")
    for g in range(lo, hi):
        first.clear()
        puct.history.clear()
        np.random.seed(g)
        torch.manual_seed(10_000 + g)
        sess = GameSession(puct, DrunkHamster(), DrunkHamster(), DrunkHamster())
        env = sess.env
        orig_reset = env.reset
        deal = {}

        def reset_and_record():
            out = orig_reset()
            deal["board"] = [[int(c) for c in r] for r in env._board]
            deal["hands"] = [[int(c) for c in h] for h in env._hands]
            return out

        env.reset = reset_and_record
        sess.play_game()
        rec = {"game": g, "board0": deal["board"], "hands0": deal["hands"],
               "results": [int(x) for x in sess.results[0]], **dict(first)}
        if MC_MAX == 20:
            rec.pop("dec", None)  # F14's record format
        recs.append(rec)
    return recs


def main():
    G = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
    W = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    t0 = time.time()
    chunks = [(G * i // W, G * (i + 1) // W) for i in range(W)]
    with mp.get_context("fork").Pool(W) as pool:
        parts = pool.map(_worker, chunks)
    games = [r for p in parts for r in p]
    res = np.array([r["results"][0] for r in games], dtype=np.float64)
    doc = {
        "protocol": f"np.random.seed(g); torch.manual_seed(10000 + g); GameSession(PUCTAgent(mc_max={MC_MAX}) with the F8 "
                    "weights (torch.manual_seed(0); PUCTAgent()), eval mode, DrunkHamster x 3).play_game(); g = 0.."
                    f"{G - 1}; seat 0's " + ("first decision" if MC_MAX == 20 else "decisions at n = 10, 6, 3 (dec[n])")
                    + ": legal cards, PUCT visit counts, chosen card",
        "deviation": "mcts.py:165-170 debug f-string removed (it raises IndexError when a legal move got no playout, "
                     "quirk Q6); the decision itself is the reference's",
        "mc_max": MC_MAX, "mc_per_card": 10, "c_puct": 2.0,
        "seat0_penalty_mean": float(-res.mean()), "seat0_penalty_sd": float(res.std(ddof=1)),
        "games": games,
    }
    with open(OUT, "w") as f:
        json.dump(doc, f)
    print(f"{G} games in {time.time() - t0:.0f}s: seat-0 penalty {-res.mean():.3f} +- {res.std(ddof=1) / np.sqrt(G):.3f}")


if __name__ == "__main__":
    main()

"""Multiplayer Elo, standing in for the third-party `multi_elo` package the
reference imports (tournament.py:5,157-164; unpinned in requirements.txt:26
and absent from this image).  PARITY UNPINNED: no reference test or fixture
records its outputs.  Restated from the published multiplayer Elo scheme
(Tom Kerrigan, "Multiplayer Elo"), which matches multi_elo's interface
`EloPlayer(place, elo)` / `calc_elo(players, k)`: every pair of players is
scored as a two-player game (1 / 0.5 / 0 by place, lower place = better)
with the usual logistic expectation, and the K factor is shared out over
the n-1 opponents.
"""


class EloPlayer:
    def __init__(self, place, elo):
        self.place = place
        self.elo = elo


def calc_elo(players, k):
    n = len(players)
    if n < 2:
        return [p.elo for p in players]
    kk = k / (n - 1)
    out = []
    for i, me in enumerate(players):
        delta = 0.0
        for j, op in enumerate(players):
            if i == j:
                continue
            actual = 1.0 if me.place < op.place else (0.5 if me.place == op.place else 0.0)
            expected = 1.0 / (1.0 + 10.0 ** ((op.elo - me.elo) / 400.0))
            delta += kk * (actual - expected)
        out.append(me.elo + delta)
    return out

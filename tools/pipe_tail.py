#!/usr/bin/env python3
"""Exact tail of the MT19937 words a pipelined k_play launch pair draws.

numpy's legacy random_interval(m) redraws masked 32-bit words until the
value is <= m, so the words one draw takes are geometric with success
probability (m + 1) / (mask + 1).  One auto-reset episode of N-player
DrunkHamster self-play draws: the deal, np.random.shuffle(arange(104)) =
random_interval(i) for i = 103..1 (env.py:99-112), and per env-step each
seat's legal[random_interval(n - 1)] for n = 10..1 (agents/random.py:9).
k_mt_ahead keeps 593..600 words twisted past the consumer position of the
launch before the running one (sechs_env.hip), so a launch PAIR must draw
<= 592 words.  A pair of 10-step launches = two episodes' draws; a pair of
5-step launches = at most one episode's (10 consecutive steps hold one deal
and every hand size once).  This prints P(words > 592) per game and launch
pair for N = 1..10 (exact convolution of the pmfs, no approximation).
"""
import numpy as np

L = 3000


def geo(m):
    d = np.zeros(L)
    if m == 0:
        d[0] = 1.0
        return d
    mask = (1 << int(m).bit_length()) - 1
    p = (m + 1) / (mask + 1)
    k = np.arange(1, L)
    d[1:] = (1 - p) ** (k - 1) * p
    return d


def conv(a, b):
    return np.convolve(a, b)[:L]


def episode_pmf(N):
    d = np.zeros(L)
    d[0] = 1.0
    for i in range(103, 0, -1):
        d = conv(d, geo(i))
    for n in range(10, 0, -1):
        for _ in range(N):
            d = conv(d, geo(n - 1))
    return d


def league_pmf(N, K, lo, hi):
    """one tournament game (league.py): the seat draw -- choice of the player
    count, permutation of the K agents -- then the episode"""
    d = episode_pmf(N)
    d = conv(d, geo(hi - lo))
    for i in range(K - 1, 0, -1):
        d = conv(d, geo(i))
    return d


def main(limit=592):
    print("N  words/episode  P(pair > %d): 10-step launches   5-step launches" % limit)
    for N in range(1, 11):
        ep = episode_pmf(N)
        two = conv(ep, ep)
        mean = (np.arange(L) * ep).sum()
        print(f"{N:2d}  {mean:13.1f}  {two[limit + 1:].sum():28.2e}  {ep[limit + 1:].sum():16.2e}")
    print("tournament handles (N = max_players, min_players 2): P(pair > %d)" % limit)
    for N, K in ((4, 5), (4, 8), (4, 16), (6, 16)):
        ep = league_pmf(N, K, 2, N)
        two = conv(ep, ep)
        print(f"  N={N} K={K:2d}: 10-step {two[limit + 1:].sum():.2e}   5-step {ep[limit + 1:].sum():.2e}")


if __name__ == "__main__":
    main()

/*
 * sechs_oracle.c -- CPU restatement of the reference 6 nimmt! hot path.
 *
 * TEST INFRASTRUCTURE ONLY (see sechs_oracle.h).  Parity pinned against the
 * reference's own outputs in tests/golden/ (tests/test_oracle_golden.py).
 *
 * Every function names the reference lines it restates.  Reference root:
 * coolo/rl-6-nimmt @ /root/reference (rl_6_nimmt/...).
 */
#include "sechs_oracle.h"

#include <stdlib.h>
#include <string.h>

/* ===================================================================== */
/* numpy legacy RandomState (MT19937).  Third-party algorithm: numpy's      */
/* legacy seeding/`random_interval` (numpy>=1.16, requirements.txt:4; the    */
/* legacy stream is frozen by numpy policy).  Pinned by golden mt19937.json */
/* ===================================================================== */
#define MT_N 624
#define MT_M 397

void or_rng_init_mt(or_rng* r, uint32_t seed) {
    /* np.random.seed(int) -> init_genrand(seed); pos = 624 */
    memset(r, 0, sizeof(*r));
    r->mode = OR_RNG_NUMPY_MT;
    r->mt[0] = seed;
    for (int i = 1; i < MT_N; i++) r->mt[i] = 1812433253u * (r->mt[i - 1] ^ (r->mt[i - 1] >> 30)) + (uint32_t)i;
    r->pos = MT_N;
}

static void mt_twist(uint32_t* mt) {
    for (int i = 0; i < MT_N; i++) {
        uint32_t y = (mt[i] & 0x80000000u) | (mt[(i + 1) % MT_N] & 0x7fffffffu);
        uint32_t v = mt[(i + MT_M) % MT_N] ^ (y >> 1);
        if (y & 1u) v ^= 0x9908b0dfu;
        mt[i] = v;
    }
}

static uint32_t mt_next(or_rng* r) {
    if (r->pos >= MT_N) {
        mt_twist(r->mt);
        r->pos = 0;
    }
    uint32_t y = r->mt[r->pos++];
    y ^= y >> 11;
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= y >> 18;
    return y;
}

/* Philox4x32-10 (Salmon et al., SC'11), the counter-based word source of  */
/* the throughput RNG mode.  Not a reference algorithm: our own stream      */
/* definition, shared by the oracle and the HIP kernels.                    */
void or_philox4x32_10(const uint32_t ctr_in[4], const uint32_t key_in[2], uint32_t out[4]) {
    uint32_t c0 = ctr_in[0], c1 = ctr_in[1], c2 = ctr_in[2], c3 = ctr_in[3];
    uint32_t k0 = key_in[0], k1 = key_in[1];
    for (int round = 0; round < 10; round++) {
        uint64_t p0 = (uint64_t)0xD2511F53u * c0;
        uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
        uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0;
        uint32_t n1 = (uint32_t)p1;
        uint32_t n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
        uint32_t n3 = (uint32_t)p0;
        c0 = n0, c1 = n1, c2 = n2, c3 = n3;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    out[0] = c0, out[1] = c1, out[2] = c2, out[3] = c3;
}

void or_rng_init_philox(or_rng* r, uint64_t seed, uint64_t stream) {
    memset(r, 0, sizeof(*r));
    r->mode = OR_RNG_PHILOX;
    r->key[0] = (uint32_t)seed;
    r->key[1] = (uint32_t)(seed >> 32);
    r->stream = stream;
    r->ctr = 0;
}

/* word w of stream s: philox(ctr = {w/4 lo, w/4 hi, s lo, s hi}, key)[w%4] */
static uint32_t philox_next(or_rng* r) {
    uint64_t blk = r->ctr >> 2;
    uint32_t ctr[4] = {(uint32_t)blk, (uint32_t)(blk >> 32), (uint32_t)r->stream, (uint32_t)(r->stream >> 32)};
    uint32_t out[4];
    or_philox4x32_10(ctr, r->key, out);
    uint32_t w = out[r->ctr & 3];
    r->ctr++;
    return w;
}

uint32_t or_rng_next(or_rng* r) { return r->mode == OR_RNG_NUMPY_MT ? mt_next(r) : philox_next(r); }

/* numpy legacy random_interval(max): masked rejection, no draw for max==0. */
uint32_t or_rng_interval(or_rng* r, uint32_t max) {
    if (max == 0) return 0;
    uint32_t mask = max;
    mask |= mask >> 1;
    mask |= mask >> 2;
    mask |= mask >> 4;
    mask |= mask >> 8;
    mask |= mask >> 16;
    uint32_t v;
    do {
        v = or_rng_next(r) & mask;
    } while (v > max);
    return v;
}

/* np.random.shuffle (legacy, 1-d array or list): Fisher-Yates from the end */
void or_shuffle_int(or_rng* r, int* a, int n) {
    for (int i = n - 1; i >= 1; i--) {
        int j = (int)or_rng_interval(r, (uint32_t)i);
        int t = a[i];
        a[i] = a[j];
        a[j] = t;
    }
}

/* ===================================================================== */
/* Rules engine: rl_6_nimmt/env.py                                         */
/* ===================================================================== */

/* env.py:224-239 _card_value */
int or_card_heads(int card) {
    int c = card + 1;
    if (c == 55) return 7;
    if (c % 11 == 0) return 5;
    if (c % 10 == 0) return 3;
    if (c % 10 == 5) return 2;
    return 1;
}

/* env.py:37 state_shape */
int or_obs_len(int include_summaries) { return 10 + 1 + (include_summaries ? 3 * OR_ROWS : 0) + OR_ROWS * OR_THRESHOLD; }

static int row_value_incl_last(const or_game* g, int r) { /* env.py:214-218 */
    int s = 0;
    for (int i = 0; i < g->row_len[r]; i++) s += or_card_heads(g->rows[r][i]);
    return s;
}

static int row_value_excl_last(const or_game* g, int r) { /* env.py:219-222 */
    int s = 0;
    for (int i = 0; i + 1 < g->row_len[r]; i++) s += or_card_heads(g->rows[r][i]);
    return s;
}

static void sort_int(int* a, int n) {
    for (int i = 1; i < n; i++)
        for (int j = i; j > 0 && a[j - 1] > a[j]; j--) {
            int t = a[j];
            a[j] = a[j - 1];
            a[j - 1] = t;
        }
}

/* env.py:99-112 _deal: hand p = sorted(deck[10p:10p+10]); row r = [deck[C-1-r]] */
void or_deal_from_deck(or_game* g, int num_players, int num_cards, const int* deck) {
    memset(g, 0, sizeof(*g));
    g->num_players = num_players;
    g->num_cards = num_cards;
    for (int p = 0; p < num_players; p++) {
        g->hand_len[p] = OR_HAND;
        for (int i = 0; i < OR_HAND; i++) g->hands[p][i] = deck[OR_HAND * p + i];
        sort_int(g->hands[p], OR_HAND);
    }
    for (int r = 0; r < OR_ROWS; r++) {
        g->row_len[r] = 1;
        g->rows[r][0] = deck[num_cards - 1 - r];
    }
}

/* env.py:43-51 reset -> _deal (np.random.shuffle(arange(C))) */
void or_reset(or_game* g, int num_players, int num_cards, or_rng* r) {
    int deck[OR_MAX_CARDS];
    for (int i = 0; i < num_cards; i++) deck[i] = i;
    or_shuffle_int(r, deck, num_cards);
    or_deal_from_deck(g, num_players, num_cards, deck);
}

/* env.py:138-152 _find_row (+ :154-159 _pick_row_to_replace) */
static int find_row(const or_game* g, int card, int* replaced) {
    int best = -1, best_last = -1, min_last = 1 << 30;
    for (int r = 0; r < OR_ROWS; r++) {
        int last = g->rows[r][g->row_len[r] - 1];
        if (last < min_last) min_last = last;
        if (last < card && last > best_last) {
            best_last = last;
            best = r;
        }
    }
    if (card < min_last) {
        /* np.argmin of row values incl. last card: first minimum wins */
        int arg = 0, val = row_value_incl_last(g, 0);
        for (int r = 1; r < OR_ROWS; r++) {
            int v = row_value_incl_last(g, r);
            if (v < val) val = v, arg = r;
        }
        *replaced = 1;
        return arg;
    }
    *replaced = 0;
    return best;
}

static int hand_find(const or_game* g, int p, int card) {
    for (int i = 0; i < g->hand_len[p]; i++)
        if (g->hands[p][i] == card) return i;
    return -1;
}

/* env.py:64-77 step -> :114-118 _check_move, :120-136 _play_cards, :161-172 _score_row */
int or_step(or_game* g, const int* actions, int32_t* rewards) {
    const int N = g->num_players;
    for (int p = 0; p < N; p++)
        if (hand_find(g, p, actions[p]) < 0) return p;
    for (int p = 0; p < N; p++) rewards[p] = 0;
    /* (card, player) sorted by card; cards are distinct */
    int order[OR_MAX_PLAYERS];
    for (int p = 0; p < N; p++) order[p] = p;
    for (int i = 1; i < N; i++)
        for (int j = i; j > 0 && actions[order[j - 1]] > actions[order[j]]; j--) {
            int t = order[j];
            order[j] = order[j - 1];
            order[j - 1] = t;
        }
    for (int k = 0; k < N; k++) {
        int p = order[k], card = actions[p], replaced;
        int r = find_row(g, card, &replaced);
        g->rows[r][g->row_len[r]++] = card; /* append (env.py:130) */
        int i = hand_find(g, p, card);      /* hands[p].remove(card) */
        for (; i + 1 < g->hand_len[p]; i++) g->hands[p][i] = g->hands[p][i + 1];
        g->hand_len[p]--;
        if (replaced || g->row_len[r] >= OR_THRESHOLD) {
            int penalty = row_value_excl_last(g, r);
            g->scores[p] += penalty;
            rewards[p] -= penalty;
            g->rows[r][0] = card;
            g->row_len[r] = 1;
        }
    }
    return -1;
}

/* env.py:246-249 */
int or_is_done(const or_game* g) { return g->hand_len[0] == 0; }

/* env.py:174-212 _create_states for one player (int64 like np.hstack) */
void or_obs(const or_game* g, int p, int include_summaries, int64_t* out) {
    int k = 0;
    for (int i = 0; i < OR_HAND; i++) out[k++] = i < g->hand_len[p] ? g->hands[p][i] : -1;
    out[k++] = g->num_players;
    if (include_summaries) {
        for (int r = 0; r < OR_ROWS; r++) out[k++] = g->row_len[r];
        for (int r = 0; r < OR_ROWS; r++) out[k++] = g->rows[r][g->row_len[r] - 1];
        for (int r = 0; r < OR_ROWS; r++) out[k++] = row_value_incl_last(g, r);
    }
    for (int r = 0; r < OR_ROWS; r++)
        for (int i = 0; i < OR_THRESHOLD; i++) out[k++] = i < g->row_len[r] ? g->rows[r][i] : -1;
}

/* agents/random.py:8-10 DrunkHamster: np.random.choice(legal) */
int or_random_policy(or_rng* r, const or_game* g, int p) {
    int n = g->hand_len[p];
    return g->hands[p][or_rng_interval(r, (uint32_t)(n - 1))];
}

/* ===================================================================== */
/* Batched self-play mirror of the sn_rollout / sn_step contract           */
/* ===================================================================== */
or_vec* or_vec_create(int B, int N, int C, int rng_mode, uint64_t seed, uint64_t game_offset) {
    or_vec* v = (or_vec*)calloc(1, sizeof(or_vec));
    v->num_games = B, v->num_players = N, v->num_cards = C, v->rng_mode = rng_mode;
    v->seed = seed, v->game_offset = game_offset;
    v->games = (or_game*)calloc((size_t)B, sizeof(or_game));
    v->rngs = (or_rng*)calloc((size_t)B, sizeof(or_rng));
    v->sum_results = (int32_t*)calloc((size_t)B * N, sizeof(int32_t));
    v->episodes = (int32_t*)calloc((size_t)B, sizeof(int32_t));
    for (int g = 0; g < B; g++) {
        uint64_t gid = game_offset + (uint64_t)g;
        if (rng_mode == OR_RNG_NUMPY_MT)
            or_rng_init_mt(&v->rngs[g], (uint32_t)(seed + gid)); /* np.random.seed(seed + g) */
        else
            or_rng_init_philox(&v->rngs[g], seed, gid);
    }
    return v;
}

void or_vec_destroy(or_vec* v) {
    if (!v) return;
    free(v->games), free(v->rngs), free(v->sum_results), free(v->episodes), free(v);
}

void or_vec_reset(or_vec* v) {
    for (int g = 0; g < v->num_games; g++) or_reset(&v->games[g], v->num_players, v->num_cards, &v->rngs[g]);
}

static void finish_episode(or_vec* v, int g) {
    or_game* G = &v->games[g];
    for (int p = 0; p < v->num_players; p++) v->sum_results[(size_t)g * v->num_players + p] -= G->scores[p];
    v->episodes[g]++;
    or_reset(G, v->num_players, v->num_cards, &v->rngs[g]); /* next GameSession.play_game() */
}

static void rollout_game(or_vec* v, int g, int steps, int summ, int32_t* rewards, uint8_t* done, uint8_t* actions,
                         int8_t* obs) {
    const int N = v->num_players, B = v->num_games, L = or_obs_len(summ);
    or_game* G = &v->games[g];
    or_rng* R = &v->rngs[g];
    int64_t o[64];
    for (int t = 0; t < steps; t++) {
        if (obs)
            for (int p = 0; p < N; p++) {
                or_obs(G, p, summ, o);
                int8_t* dst = obs + (((size_t)t * B + g) * N + p) * L;
                for (int i = 0; i < L; i++) dst[i] = (int8_t)o[i];
            }
        int a[OR_MAX_PLAYERS];
        int32_t rw[OR_MAX_PLAYERS];
        for (int p = 0; p < N; p++) a[p] = or_random_policy(R, G, p); /* agents in seat order (play.py:38-41) */
        or_step(G, a, rw);
        int d = or_is_done(G);
        if (rewards)
            for (int p = 0; p < N; p++) rewards[((size_t)t * B + g) * N + p] = rw[p];
        if (actions)
            for (int p = 0; p < N; p++) actions[((size_t)t * B + g) * N + p] = (uint8_t)a[p];
        if (done) done[(size_t)t * B + g] = (uint8_t)d;
        if (d) finish_episode(v, g);
    }
}

void or_vec_rollout(or_vec* v, int steps, int include_summaries, int32_t* rewards, uint8_t* done, uint8_t* actions,
                    int8_t* obs, int nthreads) {
#ifdef _OPENMP
#pragma omp parallel for schedule(static) num_threads(nthreads > 0 ? nthreads : 1)
#endif
    for (int g = 0; g < v->num_games; g++) rollout_game(v, g, steps, include_summaries, rewards, done, actions, obs);
    (void)nthreads;
}

int or_vec_step(or_vec* v, const int32_t* actions, int32_t* rewards, uint8_t* done, int32_t* invalid, int auto_reset) {
    const int N = v->num_players;
    int n_invalid = 0;
    for (int g = 0; g < v->num_games; g++) {
        or_game* G = &v->games[g];
        int a[OR_MAX_PLAYERS];
        int32_t rw[OR_MAX_PLAYERS] = {0};
        for (int p = 0; p < N; p++) a[p] = actions[(size_t)g * N + p];
        int bad = or_step(G, a, rw);
        invalid[g] = bad;
        if (bad >= 0) {
            n_invalid++;
            for (int p = 0; p < N; p++) rewards[(size_t)g * N + p] = 0;
            done[g] = 0;
            continue;
        }
        for (int p = 0; p < N; p++) rewards[(size_t)g * N + p] = rw[p];
        done[g] = (uint8_t)or_is_done(G);
        if (done[g] && auto_reset) finish_episode(v, g);
    }
    return n_invalid;
}

void or_vec_obs(const or_vec* v, int include_summaries, int8_t* out) {
    const int N = v->num_players, L = or_obs_len(include_summaries);
    int64_t o[64];
    for (int g = 0; g < v->num_games; g++)
        for (int p = 0; p < N; p++) {
            or_obs(&v->games[g], p, include_summaries, o);
            for (int i = 0; i < L; i++) out[((size_t)g * N + p) * L + i] = (int8_t)o[i];
        }
}

void or_vec_scores(const or_vec* v, int32_t* out) {
    for (int g = 0; g < v->num_games; g++)
        for (int p = 0; p < v->num_players; p++) out[(size_t)g * v->num_players + p] = v->games[g].scores[p];
}

/* ===================================================================== */
/* MCS agent, reference-exact: rl_6_nimmt/agents/mcts.py:17-188             */
/* ===================================================================== */
void or_mcs_init(or_mcs* m, int mc_per_card, int mc_max) {
    memset(m, 0, sizeof(*m));
    m->mc_per_card = mc_per_card;
    m->mc_max = mc_max;
}

static void avail_remove(or_mcs* m, int card) { /* list.remove, silently ignoring misses (mcts.py:70-73) */
    for (int i = 0; i < m->n_avail; i++)
        if (m->avail[i] == card) {
            for (; i + 1 < m->n_avail; i++) m->avail[i] = m->avail[i + 1];
            m->n_avail--;
            return;
        }
}

static long long factorial_capped(int n, long long cap) {
    long long f = 1;
    for (int i = 2; i <= n; i++) {
        f *= i;
        if (f > cap) return cap + 1;
    }
    return f;
}

static int mcs_forward_q6(or_mcs* m, or_rng* r, const int64_t* state, int include_summaries, const int* legal, int n,
                          int* q6) {
    const int L = or_obs_len(include_summaries);
    const int64_t* board = state + L - OR_ROWS * OR_THRESHOLD; /* _board_from_state: state[-24:] (mcts.py:75-85) */
    if (n == OR_HAND) {                                          /* _initialize_game (mcts.py:62-64) */
        m->n_avail = OR_MAX_CARDS;
        for (int i = 0; i < OR_MAX_CARDS; i++) m->avail[i] = i;
        m->num_players = (int)state[10];
    }
    /* _memorize_cards (mcts.py:66-73): legal + flattened board, negatives skipped */
    for (int i = 0; i < n; i++) avail_remove(m, legal[i]);
    for (int i = 0; i < OR_ROWS * OR_THRESHOLD; i++)
        if (board[i] >= 0) avail_remove(m, (int)board[i]);
    if (n == 1) return legal[0]; /* mcts.py:52-53 */

    /* _mcts (mcts.py:91-103), n_mc = min(mc_max, mc_per_card * n!) (:105-106) */
    long long cap = m->mc_max;
    long long f = factorial_capped(n, cap);
    long long n_mc = (long long)m->mc_per_card * f;
    if (n_mc > cap) n_mc = cap;
    double sum[OR_HAND] = {0};
    int cnt[OR_HAND] = {0};
    const int N = m->num_players;
    for (long long it = 0; it < n_mc; it++) {
        /* _draw_env + _deal_hands (mcts.py:108-127) */
        or_game g;
        memset(&g, 0, sizeof(g));
        g.num_players = N;
        g.num_cards = OR_MAX_CARDS;
        for (int rr = 0; rr < OR_ROWS; rr++) {
            g.row_len[rr] = 0;
            for (int i = 0; i < OR_THRESHOLD; i++)
                if (board[rr * OR_THRESHOLD + i] >= 0) g.rows[rr][g.row_len[rr]++] = (int)board[rr * OR_THRESHOLD + i];
        }
        g.hand_len[0] = n;
        for (int i = 0; i < n; i++) g.hands[0][i] = legal[i];
        int cards[OR_MAX_CARDS];
        for (int i = 0; i < m->n_avail; i++) cards[i] = m->avail[i];
        or_shuffle_int(r, cards, m->n_avail);
        for (int p = 1; p < N; p++) {
            g.hand_len[p] = n;
            for (int i = 0; i < n; i++) g.hands[p][i] = cards[(p - 1) * n + i];
            sort_int(g.hands[p], n);
        }
        /* _play_out (mcts.py:129-154) with MCSAgent._choose_action_mc uniform (:187-188) */
        int first = -1;
        double outcome = 0.0;
        while (!or_is_done(&g)) {
            int a[OR_MAX_PLAYERS];
            int32_t rw[OR_MAX_PLAYERS];
            for (int p = 0; p < N; p++) a[p] = or_random_policy(r, &g, p);
            if (first < 0) first = a[0];
            or_step(&g, a, rw);
            outcome += rw[0];
        }
        for (int i = 0; i < n; i++)
            if (legal[i] == first) sum[i] += outcome, cnt[i]++;
    }
    /* _choose_action_from_outcomes (mcts.py:156-172); the debug f-string at
       :170 indexes log_probs[a][0] for every action -> IndexError if any
       action got no rollout (quirk Q6): flagged in *q6, and the best mean
       over the moves that got playouts is returned (the device's choice) */
    int best = legal[0];
    double best_mean = -1.0 / 0.0;
    for (int i = 0; i < n; i++) {
        if (cnt[i] == 0) {
            *q6 = 1;
            continue;
        }
        double mean = sum[i] / (double)cnt[i];
        if (mean > best_mean) best_mean = mean, best = legal[i];
    }
    return best;
}

int or_mcs_forward(or_mcs* m, or_rng* r, const int64_t* state, int include_summaries, const int* legal, int n) {
    int q6 = 0;
    const int a = mcs_forward_q6(m, r, state, include_summaries, legal, n, &q6);
    return q6 ? -2 : a;
}

int or_mcs_game(const char* seats, int num_players, int mc_per_card, int mc_max, uint32_t seed, int* actions,
                int32_t* rewards) {
    or_rng r;
    or_rng_init_mt(&r, seed);
    or_game g;
    or_reset(&g, num_players, OR_MAX_CARDS, &r);
    or_mcs agents[OR_MAX_PLAYERS];
    for (int p = 0; p < num_players; p++) or_mcs_init(&agents[p], mc_per_card, mc_max);
    int64_t st[64];
    for (int t = 0; !or_is_done(&g); t++) {
        int a[OR_MAX_PLAYERS];
        for (int p = 0; p < num_players; p++) {
            if (seats[p] == 'M') {
                or_obs(&g, p, 1, st);
                a[p] = or_mcs_forward(&agents[p], &r, st, 1, g.hands[p], g.hand_len[p]);
                if (a[p] < 0) return -2;
            } else {
                a[p] = or_random_policy(&r, &g, p);
            }
        }
        int32_t rw[OR_MAX_PLAYERS];
        or_step(&g, a, rw);
        for (int p = 0; p < num_players; p++) actions[t * num_players + p] = a[p], rewards[t * num_players + p] = rw[p];
    }
    return 0;
}

/* ===================================================================== */
/* MCS, stratified mode: restatement of the batched engine's sampling      */
/* (mcts.py:108-154 with a fixed first move and philox words)              */
/* ===================================================================== */
int or_mcs_memorize(int* avail, int n_avail, const or_game* g, int seat, int mcs_cards) {
    or_mcs m;
    if (g->hand_len[seat] == OR_HAND) { /* _initialize_game */
        n_avail = mcs_cards;
        for (int i = 0; i < mcs_cards; i++) avail[i] = i;
    }
    m.n_avail = n_avail;
    for (int i = 0; i < n_avail; i++) m.avail[i] = avail[i];
    for (int i = 0; i < g->hand_len[seat]; i++) avail_remove(&m, g->hands[seat][i]);
    for (int r = 0; r < OR_ROWS; r++)
        for (int i = 0; i < g->row_len[r]; i++) avail_remove(&m, g->rows[r][i]);
    for (int i = 0; i < m.n_avail; i++) avail[i] = m.avail[i];
    return m.n_avail;
}

void or_mcs_stratified(const or_game* root, int seat, const int* avail, int n_avail, int rollouts, uint64_t seed,
                       uint32_t step, uint64_t gid, int32_t* sums) {
    const int N = root->num_players, n = root->hand_len[seat];
    for (int a = 0; a < OR_HAND; a++) sums[a] = 0;
    if (n <= 1) return;
    const uint64_t key = ((seed & 0xFFFFFFFF00000000ull) | (uint32_t)((uint32_t)seed ^ step));
    for (int a = 0; a < n; a++) {
        for (int r = 0; r < rollouts; r++) {
            or_rng rng;
            or_rng_init_philox(&rng, key,
                               ((uint64_t)(uint32_t)gid << 32) | ((uint64_t)seat << 24) | ((uint64_t)a << 16) | (uint64_t)r);
            /* rollout seat 0 = the decider, then the other seats in order */
            or_game g;
            memset(&g, 0, sizeof(g));
            g.num_players = N;
            g.num_cards = root->num_cards;
            for (int rr = 0; rr < OR_ROWS; rr++) {
                g.row_len[rr] = root->row_len[rr];
                for (int i = 0; i < root->row_len[rr]; i++) g.rows[rr][i] = root->rows[rr][i];
            }
            g.hand_len[0] = n;
            for (int i = 0; i < n; i++) g.hands[0][i] = root->hands[seat][i];
            int pool[OR_MAX_CARDS], left = n_avail;
            for (int i = 0; i < n_avail; i++) pool[i] = avail[i];
            for (int q = 1; q < N; q++) {
                g.hand_len[q] = 0;
                for (int i = 0; i < n && left > 0; i++) {
                    int k = (int)or_rng_interval(&rng, (uint32_t)(left - 1));
                    g.hands[q][g.hand_len[q]++] = pool[k];
                    for (int j = k; j + 1 < left; j++) pool[j] = pool[j + 1];
                    left--;
                }
                sort_int(g.hands[q], g.hand_len[q]);
            }
            int32_t outcome = 0;
            for (int t = 0; t < n; t++) {
                int acts[OR_MAX_PLAYERS];
                int32_t rw[OR_MAX_PLAYERS];
                for (int q = 0; q < N; q++) {
                    int idx = (q == 0 && t == 0) ? a : (int)or_rng_interval(&rng, (uint32_t)(g.hand_len[q] - 1));
                    acts[q] = g.hands[q][idx];
                }
                or_step(&g, acts, rw);
                outcome += rw[0];
            }
            sums[a] += outcome;
        }
    }
}

/* ===================================================================== */
/* Tournament of DrunkHamster and MCSAgent agents (tournament.py:132-177,  */
/* play.py:23-75, agents/random.py:8-10, agents/mcts.py:43-188)            */
/* ===================================================================== */
void or_league_mixed(const char* kinds, int K, int lo, int hi, const int* mc_per_card, const int* mc_max, uint64_t seed,
                     uint64_t game_offset, int slots, int games, int32_t* rec, int32_t* status, int nthreads) {
#pragma omp parallel for schedule(dynamic) num_threads(nthreads > 0 ? nthreads : 1)
    for (int j = 0; j < slots; j++) {
        or_rng r;
        or_rng_init_mt(&r, (uint32_t)(seed + game_offset + (uint64_t)j)); /* np.random.seed(seed + g) */
        status[j] = 0;
        for (int e = 0; e < games; e++) {
            /* _choose_players (tournament.py:166-177): choice(range(lo, hi + 1))
               = lo + random_interval(hi - lo); choice(K, k, replace=False) =
               permutation(K)[:k] */
            const int k = lo + (int)or_rng_interval(&r, (uint32_t)(hi - lo));
            int perm[16];
            for (int i = 0; i < K; i++) perm[i] = i;
            or_shuffle_int(&r, perm, K);
            /* GameSession(*agents).play_game(): a k-player env, reset (the deal) */
            or_game g;
            or_reset(&g, k, OR_MAX_CARDS, &r);
            or_mcs mcs[OR_MAX_PLAYERS];
            for (int p = 0; p < k; p++) or_mcs_init(&mcs[p], mc_per_card[perm[p]], mc_max[perm[p]]);
            int64_t st[64];
            while (!or_is_done(&g)) {
                int a[OR_MAX_PLAYERS];
                for (int p = 0; p < k; p++) { /* agents in seat order (play.py:38-41) */
                    if (kinds[perm[p]] == 'M') {
                        int q6 = 0;
                        or_obs(&g, p, 1, st);
                        a[p] = mcs_forward_q6(&mcs[p], &r, st, 1, g.hands[p], g.hand_len[p], &q6);
                        status[j] += q6;
                    } else {
                        a[p] = or_random_policy(&r, &g, p);
                    }
                }
                int32_t rw[OR_MAX_PLAYERS];
                or_step(&g, a, rw);
            }
            int32_t* out = rec + ((int64_t)e * slots + j) * (1 + hi);
            uint32_t w = (uint32_t)k;
            for (int p = 0; p < k; p++) w |= (uint32_t)perm[p] << (4 + 4 * p);
            out[0] = (int32_t)w;
            for (int p = 0; p < hi; p++) out[1 + p] = (p < k) ? -g.scores[p] : 0;
        }
    }
}

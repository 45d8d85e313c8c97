// sechs_mcs.h -- reference-exact MCSAgent search (agents/mcts.py:91-172) on a
// lane's numpy MT19937 stream, shared by the MCS kernels (sechs_mcs.hip) and
// the batched tournament (sechs_league.hip).
#pragma once
#include "sechs_state.h"

namespace sechs {

// ============================================================================
// reference-exact engine (numpy MT19937 streams)
// ============================================================================
// MCSAgent._mcts (mcts.py:91-106) for one decision, on this lane's stream.
// lds = this lane's 108-byte scratch.  Returns the chosen card; *q6 is set
// when some legal move got no playout (the reference then raises
// IndexError at mcts.py:170, quirk Q6; we still return the best sampled).
template <int N>
__device__ uint32_t mcs_decide_exact(MtGen& gen, ByteBuf& buf, uint8_t* lds, const Board& root, const Hand& me,
                                     uint32_t n, u32x4 avail, int mc_per_card, int mc_max, int32_t (&sum)[kHand],
                                     int32_t (&cnt)[kHand], bool* q6) {
#pragma unroll
    for (int i = 0; i < kHand; i++) sum[i] = 0, cnt[i] = 0;
    int64_t fact = 1;
    for (uint32_t i = 2; i <= n; i++) fact *= i;
    const int64_t n_mc = min((int64_t)mc_max, (int64_t)mc_per_card * fact);
    const uint32_t A = set_count(avail);
    for (int64_t it = 0; it < n_mc; it++) {
        // _deal_hands: cards = available.copy() (ascending); np.random.shuffle(cards)
        {
            uint32_t k = 0;
            const uint32_t w[4] = {avail.x, avail.y, avail.z, avail.w};
#pragma unroll
            for (int q = 0; q < 4; q++) {
                uint32_t x = w[q];
                while (x) {
                    lds[k++] = (uint8_t)(32 * q + __builtin_ctz(x));
                    x &= x - 1u;
                }
            }
        }
        for (int i = (int)A - 1; i >= 1; --i) {
            const uint32_t j = rng_interval(gen, buf, (uint32_t)i);
            const uint8_t di = lds[i], dj = lds[j];
            lds[i] = dj;
            lds[j] = di;
        }
        Game<N> R;
        R.hand[0] = me;
        R.b = root;
#pragma unroll
        for (int q = 1; q < N; q++) {
            u32x4 set = {0u, 0u, 0u, 0u};
            for (uint32_t i = 0; i < n; i++) set = set_bit(set, lds[(q - 1) * n + i]);
            R.hand[q] = hand_from_set(set);
        }
        // _play_out with uniform moves for every seat (mcts.py:129-154, :187-188)
        uint32_t first = 0;
        int32_t outcome = 0;
        for (uint32_t t = 0; t < n; t++) {
            const uint32_t cur = n - t;
            uint32_t card[N], pen[N];
#pragma unroll
            for (int q = 0; q < N; q++) {
                const uint32_t idx = rng_interval(gen, buf, cur - 1u);
                if (q == 0 && t == 0) first = idx;
                card[q] = hand_get(R.hand[q], idx);
                hand_del(R.hand[q], idx);
            }
            resolve<N>(R.b, card, pen);
            outcome -= (int32_t)pen[0];
        }
#pragma unroll
        for (int i = 0; i < kHand; i++) {
            const bool hit = (uint32_t)i == first;
            sum[i] += hit ? outcome : 0;
            cnt[i] += hit ? 1 : 0;
        }
    }
    // _choose_action_from_outcomes: best mean in legal order, strict '>'
    uint32_t best = 0;
    double best_mean = -__builtin_inf();
    bool missing = false;
#pragma unroll
    for (int i = 0; i < kHand; i++) {
        if ((uint32_t)i >= n) continue;
        if (cnt[i] == 0) {
            missing = true;  // np.mean([]) is NaN: never '>'
            continue;
        }
        const double mean = (double)sum[i] / (double)cnt[i];
        if (mean > best_mean) best_mean = mean, best = (uint32_t)i;
    }
    *q6 = missing;
    return hand_get(me, best);
}

}  // namespace sechs

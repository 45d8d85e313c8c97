// sechs_mcs_wave.h -- reference-exact MCSAgent search (agents/mcts.py:91-172)
// with one wave per decision.
//
// The lane form (sechs_mcs.h) walks one numpy MT19937 stream through every
// playout in order: its rollouts are a serial chain of ~26 k random_interval
// draws (mc_max = 200) and scattered state loads, so a league step with an
// MCS seat in every slot is bound by one lane's chain (~180 ms).  But every
// draw's maximum is known before the words are seen: the playout deal is
// np.random.shuffle of the A unseen cards (maxima A-1 .. 1), then each of
// the k seats draws legal[random_interval(cur - 1)] with cur = n - t
// (mcts.py:108-154, agents/random.py:9).  So a wave
//   (1) owns the decision's stream (the 624-word state in LDS, twisted in
//       numpy's in-place order 64 words at a time),
//   (2) decodes the draws 64 stream words per instruction -- a word's draw
//       index is its prefix count of accepted words, acceptance depends on
//       that index (numpy's masked rejection), iterated ballot -> v_mbcnt to
//       the fixed point -- for 64 playouts at a time,
//   (3) plays those 64 playouts in its 64 lanes,
// and the same words are consumed, in the same order, as by the reference.
#pragma once
#include "sechs_state.h"

namespace sechs {

constexpr uint32_t kWmStage = 1024;  // tempered low bytes staged ahead of the decoder (ring)
constexpr uint32_t kWmMaxP = 160;    // draws per playout: (A - 1) + k (n - 1) <= 102 + 6 * 9

// a numpy MT19937 stream owned by one wave: state code semantics as MtGen
// (sechs_device.h: slots [0, T) hold this round, [T, 624) the previous one;
// the stream continues with the staged words [rd, wr))
struct WaveMt {
    uint32_t* st;    // LDS [624]
    uint8_t* stage;  // LDS [kWmStage], by stream word index
    uint32_t T, rd, wr, mt0;
    bool mt0_set;
    uint32_t* head;  // LDS [64] or NULL: the previous round's slots 0..63 when a new round starts (numpy export)
};

// import a state code: the twisted-unconsumed words st[T - rem .. T) (mod
// 624: a straddling code reads the old round's tail first) are staged
__device__ __forceinline__ void wmt_load(WaveMt& m, const uint32_t* gst, uint32_t code, uint32_t lane) {
    for (uint32_t i = lane; i < (uint32_t)kMtN; i += 64u) m.st[i] = gst[i];
    __syncthreads();
    uint32_t T = code & 0x7FFu;
    if (T == 0u) T = kMtN;  // round complete: the next word twists slot 0
    const uint32_t rem = (code >> 16) & kMtCntMask;
    for (uint32_t w = lane; w < rem; w += 64u) {
        uint32_t idx = T + (uint32_t)kMtN - rem + w;
        idx = (idx >= (uint32_t)kMtN) ? idx - kMtN : idx;
        idx = (idx >= (uint32_t)kMtN) ? idx - kMtN : idx;
        m.stage[w] = (uint8_t)(mt_temper(m.st[idx]) & 0xFFu);
    }
    m.T = T, m.rd = 0u, m.wr = rem, m.mt0 = 0u, m.mt0_set = false;  // (head: the caller's)
    __syncthreads();
}

// the next <= 64 words of numpy's in-place twist (never across the round's
// end, so slot 0 of a new round is the first word of a chunk): word j reads
// old j, j + 1 and j + 397, or new j - 227 -- all read before any lane writes
__device__ __forceinline__ void wmt_twist(WaveMt& m, uint32_t lane) {
    const uint32_t S = (m.T == (uint32_t)kMtN) ? 0u : m.T;
    const uint32_t len = min(64u, (uint32_t)kMtN - S);
    const uint32_t idx = S + lane;
    uint32_t a = 0u, v = 0u;
    if (lane < len) {
        a = m.st[idx];
        const uint32_t b = m.st[(idx + 1u == (uint32_t)kMtN) ? 0u : idx + 1u];
        const uint32_t c = m.st[(idx + kMtM >= (uint32_t)kMtN) ? idx + kMtM - kMtN : idx + kMtM];
        v = mt_mix(a, b, c);
    }
    __syncthreads();
    if (S == 0u && m.head) m.head[lane] = a;
    if (lane < len) {
        m.st[idx] = v;
        m.stage[(m.wr + lane) & (kWmStage - 1u)] = (uint8_t)(mt_temper(v) & 0xFFu);
    }
    if (S == 0u) {  // slot 0's old value: the export of a straddling code needs it (mt0)
        m.mt0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)a);
        m.mt0_set = true;
    }
    m.wr += len;
    m.T = S + len;
    __syncthreads();
}

// the next `cnt` draws, draw o = random_interval(maxof(o)) (1 <= maxima <=
// 255), into out[0, cnt)
template <class MaxOf>
__device__ __forceinline__ void wmt_draws(WaveMt& m, uint32_t cnt, MaxOf maxof, uint8_t* out, uint32_t lane) {
    uint32_t o0 = 0u;
    while (o0 < cnt) {
        while (m.wr - m.rd < 64u) wmt_twist(m, lane);
        const uint32_t x = m.stage[(m.rd + lane) & (kWmStage - 1u)];
        auto eval = [&](uint32_t pre, uint32_t& mx) -> bool {
            const uint32_t o = o0 + pre;
            if (o >= cnt) {
                mx = 1u;
                return false;
            }
            mx = maxof(o);
            return (x & (0xFFFFFFFFu >> __builtin_clz(mx))) <= mx;
        };
        uint32_t mx;
        // first guess: about 3 of 4 words accepted; then to the fixed point
        uint64_t Acc = __ballot(eval((lane * 3u) >> 2, mx));
        while (true) {
            const uint32_t pre = __builtin_amdgcn_mbcnt_hi((uint32_t)(Acc >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)Acc, 0u));
            const uint64_t A2 = __ballot(eval(pre, mx));
            if (A2 == Acc) break;
            Acc = A2;
        }
        const uint32_t pre = __builtin_amdgcn_mbcnt_hi((uint32_t)(Acc >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)Acc, 0u));
        if ((Acc >> lane) & 1ull) {
            (void)eval(pre, mx);
            out[o0 + pre] = (uint8_t)(x & (0xFFFFFFFFu >> __builtin_clz(mx)));
        }
        const uint32_t na = (uint32_t)__popcll(Acc);
        if (o0 + na >= cnt) {  // the last draw is in this batch: the stream stops past its word
            m.rd += 64u - (uint32_t)__builtin_clzll(Acc);
            break;
        }
        o0 += na;
        m.rd += 64u;
    }
    __syncthreads();
}

// export: the state back in MtGen's code form (a straddle keeps old slot 0 in mt0)
__device__ __forceinline__ void wmt_store(const WaveMt& m, uint32_t* gst, uint32_t* code, uint32_t* mt0, uint32_t lane) {
    for (uint32_t i = lane; i < (uint32_t)kMtN; i += 64u) gst[i] = m.st[i];
    if (lane == 0u) {
        *code = m.T | ((m.wr - m.rd) << 16);
        if (m.mt0_set) *mt0 = m.mt0;
    }
}

// export in numpy's (key, pos) form: a consumer still in the previous round
// (the stream ran at most one 64-word chunk into the next) gets that round's
// key back from the saved head; otherwise the current round is finished in
// place, as numpy twists whole blocks (mt_export, sechs_mcs.hip)
__device__ __forceinline__ int32_t wmt_store_numpy(WaveMt& m, uint32_t* key, uint32_t lane) {
    const uint32_t u = m.wr - m.rd;  // staged, unconsumed
    if (m.head && u > m.T) {         // straddle: T <= 64
        for (uint32_t i = lane; i < (uint32_t)kMtN; i += 64u) key[i] = (i < m.T) ? m.head[i] : m.st[i];
        return (int32_t)(kMtN - (u - m.T));
    }
    const uint32_t pos = m.T - u;
    while (m.T < (uint32_t)kMtN) wmt_twist(m, lane);
    for (uint32_t i = lane; i < (uint32_t)kMtN; i += 64u) key[i] = m.st[i];
    return (int32_t)pos;
}

// One playout (mcts.py:108-154) from its decoded draws d: shuffle the unseen
// cards (ascending, `sorted`) in this lane's deck, deal the k-1 opponents n
// cards each, play n rounds with uniform moves for every seat.
template <int K>
__device__ __forceinline__ void wmcs_playout(const uint8_t* d, uint32_t A, uint32_t n, const uint8_t* sorted, uint8_t* deck,
                                             const Board& root, const Hand& me, int32_t (&sum)[kHand],
                                             int32_t (&cnt)[kHand]) {
    for (uint32_t i = 0; i < A; i += 4u) *(uint32_t*)(deck + i) = *(const uint32_t*)(sorted + i);
    for (int i = (int)A - 1; i >= 1; --i) {
        const uint32_t j = d[A - 1u - (uint32_t)i];
        const uint8_t di = deck[i], dj = deck[j];
        deck[i] = dj;
        deck[j] = di;
    }
    Game<K> R;
    R.hand[0] = me;
    R.b = root;
#pragma unroll
    for (int q = 1; q < K; q++) {
        u32x4 set = {0u, 0u, 0u, 0u};
        for (uint32_t i = 0; i < n; i++) set = set_bit(set, deck[(q - 1) * n + i]);
        R.hand[q] = hand_from_set(set);
    }
    const uint8_t* dp = d + (A - 1u);
    uint32_t first = 0;
    int32_t outcome = 0;
    for (uint32_t t = 0; t < n; t++) {
        uint32_t card[K], pen[K];
#pragma unroll
        for (int q = 0; q < K; q++) {
            const uint32_t idx = (t + 1u < n) ? dp[t * K + q] : 0u;  // random_interval(0): no draw
            if (q == 0 && t == 0) first = idx;
            card[q] = hand_get(R.hand[q], idx);
            hand_del(R.hand[q], idx);
        }
        resolve<K>(R.b, card, pen);
        outcome -= (int32_t)pen[0];
    }
#pragma unroll
    for (int i = 0; i < kHand; i++) {
        const bool hit = (uint32_t)i == first;
        sum[i] += hit ? outcome : 0;
        cnt[i] += hit ? 1 : 0;
    }
}

// LDS a decision wave needs
struct WmcsLds {
    uint32_t st[kMtN];
    uint8_t stage[kWmStage];
    uint8_t dr[64 * kWmMaxP];
    uint8_t deck[64 * kDeckStride];
    uint8_t sorted[kDeckStride];
};

// MCSAgent._mcts + _choose_action_from_outcomes (mcts.py:91-106, 156-172) for
// a game of K players, on the wave's stream: the chosen card; *q6 when some
// legal move got no playout (the reference raises IndexError, quirk Q6)
// (inlined into the league step kernel: there the stream cursor, the card
// memory and the hands then stay in registers -- 225 -> 138 VGPRs, league MCS
// step 164 -> 106 ms per run.py round; the one-decision drop-in kernel keeps
// the out-of-line form, wmcs_decide below)
template <int K>
__device__ __forceinline__ uint32_t wmcs_decide_inl(WaveMt& m, WmcsLds& L, const Board& root, const Hand& me, uint32_t n,
                                                    u32x4 avail, int mc_per_card, int mc_max, bool* q6, uint32_t lane,
                                                    int32_t* sums_out = nullptr, int32_t* counts_out = nullptr) {
    int64_t fact = 1;
    for (uint32_t i = 2; i <= n; i++) fact *= i;
    const uint32_t n_mc = (uint32_t)min((int64_t)mc_max, (int64_t)mc_per_card * fact);
    const uint32_t A = set_count(avail), A1 = A - 1u, n1 = n - 1u;
    const uint32_t P = A1 + (uint32_t)K * n1;  // draws per playout
    const uint32_t magic = (uint32_t)((0x100000000ull + P - 1u) / P);       // o / P for o < 2^32 / P
    const uint32_t invk = (65536u + (uint32_t)K - 1u) / (uint32_t)K;        // q / K for q < 65536 / K
    if (lane == 0u) {  // cards = available.copy() (ascending)
        uint32_t k = 0;
        const uint32_t w[4] = {avail.x, avail.y, avail.z, avail.w};
        for (int q = 0; q < 4; q++) {
            uint32_t x = w[q];
            while (x) {
                L.sorted[k++] = (uint8_t)(32 * q + __builtin_ctz(x));
                x &= x - 1u;
            }
        }
    }
    __syncthreads();
    int32_t sum[kHand], cnt[kHand];
#pragma unroll
    for (int i = 0; i < kHand; i++) sum[i] = 0, cnt[i] = 0;
    for (uint32_t r0 = 0; r0 < n_mc; r0 += 64u) {
        const uint32_t nb = min(64u, n_mc - r0);
        wmt_draws(
            m, nb * P,
            [&](uint32_t o) -> uint32_t {
                const uint32_t r = __umulhi(o, magic), orr = o - r * P;
                return (orr < A1) ? A1 - orr : n1 - (__umul24(orr - A1, invk) >> 16);
            },
            L.dr, lane);
        if (lane < nb)
            wmcs_playout<K>(L.dr + lane * P, A, n, L.sorted, L.deck + lane * kDeckStride, root, me, sum, cnt);
        __syncthreads();
    }
#pragma unroll
    for (int i = 0; i < kHand; i++) {  // integer sums: any order
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) {
            sum[i] += __shfl_xor(sum[i], off);
            cnt[i] += __shfl_xor(cnt[i], off);
        }
    }
    if (lane == 0u) {
#pragma unroll
        for (int i = 0; i < kHand; i++) {
            if (sums_out) sums_out[i] = sum[i];
            if (counts_out) counts_out[i] = cnt[i];
        }
    }
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

template <int K>
__device__ uint32_t wmcs_decide(WaveMt& m, WmcsLds& L, const Board& root, const Hand& me, uint32_t n, u32x4 avail,
                                int mc_per_card, int mc_max, bool* q6, uint32_t lane, int32_t* sums_out = nullptr,
                                int32_t* counts_out = nullptr) {
    return wmcs_decide_inl<K>(m, L, root, me, n, avail, mc_per_card, mc_max, q6, lane, sums_out, counts_out);
}

}  // namespace sechs

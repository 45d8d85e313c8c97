// sechs_device.h -- per-lane 6 nimmt! game engine for gfx950 (CDNA4).
//
// One lane = one game.  Everything a step touches lives in VGPRs:
//   * a hand is a 128-bit card set (4 x u32), so the reference's sorted
//     `legal_actions` list (env.py:209) is the set bits in ascending order,
//     `card in hand` (env.py:117) is a bit test and `hands[p].remove(card)`
//     (env.py:131) is a bit clear;
//   * a row is two u32: `lo` = cards 0..3 (bytes), `hi` = card 4 | len << 8 |
//     heads << 16 | end << 24, where heads = bull heads of the whole row
//     (env.py:214-218 with include_last=True) and end = the last card
//     (env.py:140).  Bytes past `len` are kept zero.
// Rules restated from env.py:120-172.  The
// kernels never call the oracle; they are checked against it in tests/.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace sechs {

constexpr int kRows = 4;
constexpr int kThreshold = 6;
constexpr int kHand = 10;
constexpr int kMaxPlayers = 10;
constexpr int kMaxCards = 104;
constexpr int kMtN = 624;
constexpr int kMtM = 397;

enum RngMode { RNG_PHILOX = 0, RNG_NUMPY_MT = 1 };

// --------------------------------------------------------------------------
// bull heads, env.py:224-239
// --------------------------------------------------------------------------
__device__ __forceinline__ uint32_t heads_of(uint32_t c) {
    uint32_t c1 = c + 1u;
    uint32_t h = 1u;
    h = (c1 % 10u == 5u) ? 2u : h;
    h = (c1 % 10u == 0u) ? 3u : h;
    h = (c1 % 11u == 0u) ? 5u : h;
    h = (c1 == 55u) ? 7u : h;
    return h;
}

// --------------------------------------------------------------------------
// 128-bit card sets
// --------------------------------------------------------------------------
struct Hand {
    uint32_t w[4];
};

__device__ __forceinline__ void hand_clear(Hand& h) { h.w[0] = h.w[1] = h.w[2] = h.w[3] = 0u; }

__device__ __forceinline__ void hand_add(Hand& h, uint32_t c) {
    uint32_t bit = 1u << (c & 31u), q = c >> 5;
#pragma unroll
    for (int i = 0; i < 4; i++) h.w[i] |= (q == (uint32_t)i) ? bit : 0u;
}

__device__ __forceinline__ void hand_remove(Hand& h, uint32_t c) {
    uint32_t bit = 1u << (c & 31u), q = c >> 5;
#pragma unroll
    for (int i = 0; i < 4; i++) h.w[i] &= (q == (uint32_t)i) ? ~bit : 0xFFFFFFFFu;
}

__device__ __forceinline__ bool hand_has(const Hand& h, uint32_t c) {
    uint32_t q = c >> 5;
    uint32_t w = h.w[0];
    w = (q == 1u) ? h.w[1] : w;
    w = (q == 2u) ? h.w[2] : w;
    w = (q == 3u) ? h.w[3] : w;
    return (c < 128u) && ((w >> (c & 31u)) & 1u);
}

__device__ __forceinline__ uint32_t hand_count(const Hand& h) {
    return __popc(h.w[0]) + __popc(h.w[1]) + __popc(h.w[2]) + __popc(h.w[3]);
}

// position of the k-th (0-based) set bit of a 32-bit word (must exist)
__device__ __forceinline__ uint32_t select32(uint32_t w, uint32_t k) {
    uint32_t pos = 0, c;
    c = __popc(w & 0xFFFFu);
    if (k >= c) { k -= c; pos += 16; w >>= 16; }
    c = __popc(w & 0xFFu);
    if (k >= c) { k -= c; pos += 8; w >>= 8; }
    c = __popc(w & 0xFu);
    if (k >= c) { k -= c; pos += 4; w >>= 4; }
    c = __popc(w & 0x3u);
    if (k >= c) { k -= c; pos += 2; w >>= 2; }
    c = w & 1u;
    if (k >= c) pos += 1;
    return pos;
}

// k-th smallest card of the hand == legal_actions[k]
__device__ __forceinline__ uint32_t hand_select(const Hand& h, uint32_t k) {
    uint32_t c0 = __popc(h.w[0]), c1 = __popc(h.w[1]), c2 = __popc(h.w[2]);
    uint32_t w = h.w[0], base = 0;
    if (k >= c0) { k -= c0; w = h.w[1]; base = 32;
        if (k >= c1) { k -= c1; w = h.w[2]; base = 64;
            if (k >= c2) { k -= c2; w = h.w[3]; base = 96; } } }
    return base + select32(w, k);
}

// smallest card, and remove it (hand must be non-empty)
__device__ __forceinline__ uint32_t hand_pop_min(Hand& h) {
    uint32_t c;
    if (h.w[0]) { c = __builtin_ctz(h.w[0]); h.w[0] &= h.w[0] - 1u; }
    else if (h.w[1]) { c = 32 + __builtin_ctz(h.w[1]); h.w[1] &= h.w[1] - 1u; }
    else if (h.w[2]) { c = 64 + __builtin_ctz(h.w[2]); h.w[2] &= h.w[2] - 1u; }
    else { c = 96 + __builtin_ctz(h.w[3]); h.w[3] &= h.w[3] - 1u; }
    return c;
}

// --------------------------------------------------------------------------
// board rows
// --------------------------------------------------------------------------
struct Board {
    uint32_t lo[kRows];  // cards 0..3 of each row
    uint32_t hi[kRows];  // card4 | len << 8 | heads << 16 | end << 24
};

__device__ __forceinline__ uint32_t row_len(const Board& b, int r) { return (b.hi[r] >> 8) & 0xFFu; }
__device__ __forceinline__ uint32_t row_heads(const Board& b, int r) { return (b.hi[r] >> 16) & 0xFFu; }
__device__ __forceinline__ uint32_t row_end(const Board& b, int r) { return b.hi[r] >> 24; }

__device__ __forceinline__ void row_start(Board& b, int r, uint32_t c) {
    b.lo[r] = c;
    b.hi[r] = (1u << 8) | (heads_of(c) << 16) | (c << 24);
}

// card of row r at position i (i < len)
__device__ __forceinline__ uint32_t row_card(const Board& b, int r, int i) {
    return i < 4 ? (b.lo[r] >> (8 * i)) & 0xFFu : b.hi[r] & 0xFFu;
}

// --------------------------------------------------------------------------
// simultaneous play resolution, env.py:120-172.  card[p] must be legal.
// pen[p] receives the bull heads seat p takes (reward = -pen).
// --------------------------------------------------------------------------
template <int N>
__device__ __forceinline__ void resolve(Board& b, const uint32_t (&card)[N], uint32_t (&pen)[N]) {
    // (card, player) ascending by card (env.py:124-125); cards are distinct
    uint32_t key[N];
#pragma unroll
    for (int p = 0; p < N; p++) { key[p] = (card[p] << 4) | (uint32_t)p; pen[p] = 0u; }
#pragma unroll
    for (int i = 0; i < N; i++)
#pragma unroll
        for (int j = 0; j + 1 < N - i; j++) {
            uint32_t lo = min(key[j], key[j + 1]), hi = max(key[j], key[j + 1]);
            key[j] = lo, key[j + 1] = hi;
        }
#pragma unroll
    for (int k = 0; k < N; k++) {
        const uint32_t c = key[k] >> 4, p = key[k] & 15u;
        // _find_row: the row whose last card is the largest one below c
        int best = -1;
        uint32_t best_end = 0u;
#pragma unroll
        for (int r = 0; r < kRows; r++) {
            uint32_t e = row_end(b, r);
            bool ok = (e < c) && (best < 0 || e > best_end);
            best = ok ? r : best;
            best_end = ok ? e : best_end;
        }
        // undercut: _pick_row_to_replace = argmin row value, first minimum
        int minr = 0;
        uint32_t minh = row_heads(b, 0);
#pragma unroll
        for (int r = 1; r < kRows; r++) {
            uint32_t h = row_heads(b, r);
            bool lt = h < minh;
            minr = lt ? r : minr;
            minh = lt ? h : minh;
        }
        const bool under = best < 0;
        const int tr = under ? minr : best;
        const uint32_t hc = heads_of(c);
        uint32_t penalty = 0u;
#pragma unroll
        for (int r = 0; r < kRows; r++) {
            if (r == tr) {
                const uint32_t len = row_len(b, r);
                const bool take = under || len == (uint32_t)(kThreshold - 1);
                penalty = take ? row_heads(b, r) : 0u;  // _score_row: whole old row
                uint32_t lo_app = b.lo[r] | (len < 4u ? (c << (8u * len)) : 0u);
                uint32_t hi_app = (len == 4u ? c : (b.hi[r] & 0xFFu)) | ((len + 1u) << 8) |
                                  ((row_heads(b, r) + hc) << 16) | (c << 24);
                b.lo[r] = take ? c : lo_app;
                b.hi[r] = take ? ((1u << 8) | (hc << 16) | (c << 24)) : hi_app;
            }
        }
#pragma unroll
        for (int q = 0; q < N; q++) pen[q] += (p == (uint32_t)q) ? penalty : 0u;
    }
}

// --------------------------------------------------------------------------
// Random word sources.  Both feed numpy's legacy masked-rejection
// random_interval; only the 32-bit word stream differs.
// --------------------------------------------------------------------------
__device__ __forceinline__ uint32_t mt_temper(uint32_t y) {
    y ^= y >> 11;
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= y >> 18;
    return y;
}

// numpy legacy MT19937 with the twist done lazily, one word per draw, in
// place.  pos < 624: "lazy" -- words [0,pos) already hold this round's
// values, [pos,624) the previous round's; pos >= 624: "direct" -- the
// array is a fully twisted round (as np.random.get_state() returns it) and
// pos-624 is the next word to hand out.
struct MtRng {
    uint32_t* st;  // this game's 624 words
    uint32_t pos;
    __device__ __forceinline__ uint32_t next() {
        uint32_t v;
        if (pos >= (uint32_t)kMtN) {
            v = st[pos - kMtN];
            pos = (pos + 1u == 2u * kMtN) ? 0u : pos + 1u;
        } else {
            const uint32_t i = pos;
            const uint32_t i1 = (i == kMtN - 1) ? 0u : i + 1u;
            const uint32_t im = (i < (uint32_t)(kMtN - kMtM)) ? i + kMtM : i - (kMtN - kMtM);
            const uint32_t a = st[i], b = st[i1], c = st[im];
            const uint32_t y = (a & 0x80000000u) | (b & 0x7fffffffu);
            v = c ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
            st[i] = v;
            pos = i1;
        }
        return mt_temper(v);
    }
};

__device__ __forceinline__ void philox4x32_10(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0,
                                              uint32_t k1, uint32_t (&o)[4]) {
#pragma unroll
    for (int r = 0; r < 10; r++) {
        uint32_t lo0 = 0xD2511F53u * c0, hi0 = __umulhi(0xD2511F53u, c0);
        uint32_t lo1 = 0xCD9E8D57u * c2, hi1 = __umulhi(0xCD9E8D57u, c2);
        uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
        c0 = n0, c1 = lo1, c2 = n2, c3 = lo0;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    o[0] = c0, o[1] = c1, o[2] = c2, o[3] = c3;
}

// counter-based stream: word w of game s = philox({w/4, s}, seed)[w % 4]
struct PhiloxRng {
    uint32_t k0, k1, s0, s1;
    uint64_t ctr;
    uint32_t buf[4];
    __device__ __forceinline__ void refill() {
        uint64_t blk = ctr >> 2;
        philox4x32_10((uint32_t)blk, (uint32_t)(blk >> 32), s0, s1, k0, k1, buf);
    }
    __device__ __forceinline__ uint32_t next() {
        uint32_t j = (uint32_t)ctr & 3u;
        if (j == 0u) refill();
        uint32_t v = buf[0];
        v = (j == 1u) ? buf[1] : v;
        v = (j == 2u) ? buf[2] : v;
        v = (j == 3u) ? buf[3] : v;
        ctr++;
        return v;
    }
};

// numpy legacy random_interval(max)
template <class R>
__device__ __forceinline__ uint32_t rng_interval(R& r, uint32_t max) {
    if (max == 0u) return 0u;
    const uint32_t mask = 0xFFFFFFFFu >> __builtin_clz(max);
    uint32_t v;
    do {
        v = r.next() & mask;
    } while (v > max);
    return v;
}

}  // namespace sechs

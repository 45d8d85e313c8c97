// sechs_device.h -- per-lane 6 nimmt! game engine for gfx950 (CDNA4).
//
// One lane = one game; everything a step touches lives in VGPRs:
//   * a hand is the reference's sorted `legal_actions` list (env.py:209)
//     as 12 bytes {u64 lo = cards 0..7, u32 hi = cards 8..11}, ascending,
//     padded with 0xFF.  DrunkHamster's `legal[k]` (agents/random.py:9) is
//     a byte extract, `hands[p].remove(card)` (env.py:131) a byte delete,
//     and the observation's hand field (env.py:210) is the bytes as stored.
//   * the board is two 4-vectors: lo[r] = cards 0..3 of row r (bytes),
//     hi[r] = card4 | len << 8 | heads << 16 | end << 24, heads = bull heads
//     of the whole row (env.py:214-218, include_last=True), end = last card
//     (env.py:140).  Bytes past `len` are zero.
// Rules restated from env.py:120-172.  Small arrays
// that are indexed with run-time values are vector types on purpose: LLVM
// keeps those in registers, whereas plain arrays indexed that way end up in
// scratch memory.  The kernels never call the oracle; tests/ compare them.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace sechs {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// SECHS_DEBUG (the libsechs_debug.so variant, make libsechs_debug.so):
// SN_DASSERT counts violated invariants of the game engine in a device word
// (sn_debug_failures reads and clears it) instead of trapping -- a trap on a
// shared GPU box can take the queue down.  Active in sechs_env.hip's kernels
// (SECHS_DEBUG_HERE); a no-op in the product library and in the other files.
#if defined(SECHS_DEBUG) && defined(SECHS_DEBUG_HERE)
__device__ unsigned int g_sn_dbg[2] = {0u, 0xFFFFFFFFu};  // failures, first failing line
#define SN_DASSERT(c)                                                   \
    do {                                                                \
        if (!(c)) {                                                     \
            atomicAdd(&::sechs::g_sn_dbg[0], 1u);                       \
            atomicMin(&::sechs::g_sn_dbg[1], (unsigned int)__LINE__);   \
        }                                                               \
    } while (0)
#else
#define SN_DASSERT(c) ((void)0)
#endif

constexpr int kRows = 4;
constexpr int kThreshold = 6;
constexpr int kHand = 10;
constexpr int kMaxPlayers = 10;
constexpr int kMaxCards = 104;
constexpr int kMtN = 624;
constexpr int kMtM = 397;

// RNG_NUMPY_RING(_HBM): numpy-MT words pre-twisted by k_mt_prep, read from
// an LDS copy of the ring (or straight from HBM when LDS is short); k_play only
// RNG_NUMPY_PIPE: numpy-MT words twisted ahead by k_mt_ahead (the pipelined ring); k_play only
// RNG_NUMPY_DEC: decode-ahead records (k_decode decoded the draws and the deals from the pipelined ring); k_play only
enum RngMode { RNG_PHILOX = 0, RNG_NUMPY_MT = 1, RNG_NUMPY_RING = 2, RNG_NUMPY_RING_HBM = 3, RNG_NUMPY_PIPE = 4,
               RNG_NUMPY_DEC = 5 };

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
// 128-bit card sets (deal construction, card memory)
// --------------------------------------------------------------------------
__device__ __forceinline__ u32x4 set_bit(u32x4 s, uint32_t c) {
    const uint32_t bit = 1u << (c & 31u), q = c >> 5;
    s.x |= (q == 0u) ? bit : 0u;
    s.y |= (q == 1u) ? bit : 0u;
    s.z |= (q == 2u) ? bit : 0u;
    s.w |= (q == 3u) ? bit : 0u;
    return s;
}

__device__ __forceinline__ bool has_bit(u32x4 s, uint32_t c) {
    const uint32_t q = c >> 5, sh = c & 31u;
    const uint32_t w = (q == 0u) ? s.x : (q == 1u) ? s.y : (q == 2u) ? s.z : s.w;
    return (w >> sh) & 1u;
}

__device__ __forceinline__ uint32_t set_count(u32x4 s) { return __popc(s.x) + __popc(s.y) + __popc(s.z) + __popc(s.w); }

// --------------------------------------------------------------------------
// sorted hands as byte lists
// --------------------------------------------------------------------------
struct Hand {
    uint64_t lo;  // cards 0..7
    uint32_t hi;  // cards 8..9, bytes 10..11 = 0xFF
};

// legal_actions[k]
__device__ __forceinline__ uint32_t hand_get(const Hand& h, uint32_t k) {
    const uint32_t a = (uint32_t)(h.lo >> ((8u * k) & 63u));
    const uint32_t b = h.hi >> ((8u * (k - 8u)) & 31u);
    return (k < 8u ? a : b) & 0xFFu;
}

// hands[p].remove(legal_actions[k])
__device__ __forceinline__ void hand_del(Hand& h, uint32_t k) {
    const uint64_t m = (k < 8u) ? ((1ull << (8u * k)) - 1ull) : ~0ull;
    const uint64_t lo_del = (h.lo & m) | ((h.lo >> 8) & ~m) | ((uint64_t)(h.hi & 0xFFu) << 56);
    const uint32_t m2 = (k < 8u) ? 0u : ((k >= 12u) ? ~0u : ((1u << (8u * (k - 8u))) - 1u));
    const uint32_t hi_del = (h.hi & m2) | ((h.hi >> 8) & ~m2) | 0xFF000000u;
    h.lo = (k < 8u) ? lo_del : h.lo;
    h.hi = hi_del;
}

// index of card c in the hand, or -1 (SWAR zero-byte search; the lowest
// flagged byte of the classic test is exact)
__device__ __forceinline__ int hand_find(const Hand& h, uint32_t c) {
    if (c > 0xFEu) return -1;
    const uint64_t x = h.lo ^ (0x0101010101010101ull * (uint64_t)c);
    const uint64_t z = (x - 0x0101010101010101ull) & ~x & 0x8080808080808080ull;
    const uint32_t y = h.hi ^ (0x01010101u * c);
    const uint32_t zy = (y - 0x01010101u) & ~y & 0x80808080u;
    if (z) return (int)(__builtin_ctzll(z) >> 3);
    if (zy) return 8 + (int)(__builtin_ctz(zy) >> 3);
    return -1;
}

// number of cards (first 0xFF byte)
__device__ __forceinline__ uint32_t hand_len(const Hand& h) {
    const uint64_t x = ~h.lo;  // 0xFF bytes -> zero bytes
    const uint64_t z = (x - 0x0101010101010101ull) & ~x & 0x8080808080808080ull;
    const uint32_t y = ~h.hi;
    const uint32_t zy = (y - 0x01010101u) & ~y & 0x80808080u;
    return z ? (uint32_t)(__builtin_ctzll(z) >> 3) : 8u + (uint32_t)(__builtin_ctz(zy | 0x80000000u) >> 3);
}

// the listed cards strictly ascend (distinct cards; debug checks only)
__device__ __forceinline__ bool hand_strict(const Hand& h) {
    bool ok = true;
#pragma unroll
    for (uint32_t k = 0; k + 1 < (uint32_t)kHand; k++) {
        const uint32_t a = hand_get(h, k), b = hand_get(h, k + 1u);
        ok = ok && (b == 0xFFu || a < b);
    }
    return ok;
}

// sorted byte list from a card set of at most 10 cards
__device__ __forceinline__ Hand hand_from_set(u32x4 s) {
    Hand h;
    h.lo = ~0ull;
    h.hi = ~0u;
    uint32_t w0 = s.x, w1 = s.y, w2 = s.z, w3 = s.w;
#pragma unroll
    for (int k = 0; k < kHand; k++) {
        uint32_t c;
        if (w0) { c = __builtin_ctz(w0); w0 &= w0 - 1u; }
        else if (w1) { c = 32u + __builtin_ctz(w1); w1 &= w1 - 1u; }
        else if (w2) { c = 64u + __builtin_ctz(w2); w2 &= w2 - 1u; }
        else if (w3) { c = 96u + __builtin_ctz(w3); w3 &= w3 - 1u; }
        else c = 0xFFu;
        if (k < 8) h.lo = (h.lo & ~(0xFFull << (8 * k))) | ((uint64_t)c << (8 * k));
        else h.hi = (h.hi & ~(0xFFu << (8 * (k - 8)))) | (c << (8 * (k - 8)));
    }
    return h;
}

// --------------------------------------------------------------------------
// board rows
// --------------------------------------------------------------------------
struct Board {
    u32x4 lo;  // cards 0..3 of each row
    u32x4 hi;  // card4 | len << 8 | heads << 16 | end << 24
};

__device__ __forceinline__ uint32_t meta_row(uint32_t c) { return (1u << 8) | (heads_of(c) << 16) | (c << 24); }
__device__ __forceinline__ uint32_t len_of(uint32_t hi) { return (hi >> 8) & 0xFFu; }
__device__ __forceinline__ uint32_t heads_in(uint32_t hi) { return (hi >> 16) & 0xFFu; }
__device__ __forceinline__ uint32_t end_of(uint32_t hi) { return hi >> 24; }

// card i (0..4) of a row given its two words
__device__ __forceinline__ uint32_t card_at(uint32_t lo, uint32_t hi, int i) {
    return i < 4 ? (lo >> (8 * i)) & 0xFFu : hi & 0xFFu;
}

// place card c on the board (env.py:127-134 for one card); returns the
// bull heads its player takes.  info (the drop-in env's debug trace,
// env.py:128,145,165): target row | undercut << 2 | scored << 3
__device__ __forceinline__ uint32_t place_card(Board& b, uint32_t c, uint32_t* info = nullptr) {
    const uint32_t h[4] = {b.hi.x, b.hi.y, b.hi.z, b.hi.w};
    // _find_row: the row whose last card is the largest one below c
    int best = -1;
    uint32_t best_end = 0u;
#pragma unroll
    for (int r = 0; r < kRows; r++) {
        const uint32_t e = end_of(h[r]);
        const bool ok = (e < c) && (best < 0 || e > best_end);
        best = ok ? r : best;
        best_end = ok ? e : best_end;
    }
    // undercut: _pick_row_to_replace = np.argmin(row values), first minimum
    int minr = 0;
    uint32_t minh = heads_in(h[0]);
#pragma unroll
    for (int r = 1; r < kRows; r++) {
        const uint32_t v = heads_in(h[r]);
        const bool lt = v < minh;
        minr = lt ? r : minr;
        minh = lt ? v : minh;
    }
    const bool under = best < 0;
    const int tr = under ? minr : best;
    const uint32_t hc = heads_of(c);
    const uint32_t lo_t = (tr == 0) ? b.lo.x : (tr == 1) ? b.lo.y : (tr == 2) ? b.lo.z : b.lo.w;
    const uint32_t hi_t = (tr == 0) ? h[0] : (tr == 1) ? h[1] : (tr == 2) ? h[2] : h[3];
    const uint32_t len = len_of(hi_t);
    const bool take = under || len == (uint32_t)(kThreshold - 1);  // 6th card, env.py:133
    const uint32_t penalty = take ? heads_in(hi_t) : 0u;           // _score_row: the whole old row
    if (info) *info = (uint32_t)tr | (under ? 4u : 0u) | (take ? 8u : 0u);
    SN_DASSERT(c < (uint32_t)kMaxCards && len >= 1u && len <= (uint32_t)(kThreshold - 1));  // a legal card; rows hold 1..5
    SN_DASSERT(under || end_of(hi_t) < c);                                                  // the row ends below the card
    const uint32_t lo_new = take ? c : (lo_t | (len < 4u ? (c << (8u * len)) : 0u));
    const uint32_t hi_new = take ? ((1u << 8) | (hc << 16) | (c << 24))
                                 : ((len == 4u ? c : (hi_t & 0xFFu)) | ((len + 1u) << 8) |
                                    ((heads_in(hi_t) + hc) << 16) | (c << 24));
    b.lo.x = (tr == 0) ? lo_new : b.lo.x;
    b.lo.y = (tr == 1) ? lo_new : b.lo.y;
    b.lo.z = (tr == 2) ? lo_new : b.lo.z;
    b.lo.w = (tr == 3) ? lo_new : b.lo.w;
    b.hi.x = (tr == 0) ? hi_new : b.hi.x;
    b.hi.y = (tr == 1) ? hi_new : b.hi.y;
    b.hi.z = (tr == 2) ? hi_new : b.hi.z;
    b.hi.w = (tr == 3) ? hi_new : b.hi.w;
    return penalty;
}

// simultaneous play, env.py:120-136: cards in ascending order, each placed
// in turn.  card[p] must be legal.  pen[p] = bull heads seat p takes.
// SKIP: seats whose card is 0xFF (absent: a tournament game with fewer
// players than the handle's seats) play nothing.
template <int N, bool SKIP = false>
__device__ __forceinline__ void resolve(Board& b, const uint32_t (&card)[N], uint32_t (&pen)[N],
                                        uint32_t* trace = nullptr) {
    uint32_t key[N];
#pragma unroll
    for (int p = 0; p < N; p++) key[p] = (card[p] << 4) | (uint32_t)p;
#pragma unroll
    for (int i = 0; i < N; i++)
#pragma unroll
        for (int j = 0; j + 1 < N - i; j++) {
            const uint32_t lo = min(key[j], key[j + 1]), hi = max(key[j], key[j + 1]);
            key[j] = lo, key[j + 1] = hi;
        }
#pragma unroll
    for (int p = 0; p < N; p++) pen[p] = 0u;
#pragma unroll
    for (int k = 0; k + 1 < N; k++) SN_DASSERT((key[k] >> 4) < (key[k + 1] >> 4) || (key[k] >> 4) == 0xFFu);  // distinct cards
#pragma unroll
    for (int k = 0; k < N; k++) {
        if (SKIP && (key[k] >> 4) >= 0xFFu) break;  // absent seats sort last
        uint32_t info = 0u;
        const uint32_t penalty = place_card(b, key[k] >> 4, trace ? &info : nullptr);
        const uint32_t p = key[k] & 15u;
        if (trace) trace[p] = info | (penalty << 8);  // per seat: its card's row, flags, penalty
#pragma unroll
        for (int q = 0; q < N; q++) pen[q] += (p == (uint32_t)q) ? penalty : 0u;
    }
}

// --------------------------------------------------------------------------
// card-set helpers (MCS / PUCT card memory and opponent deals)
// --------------------------------------------------------------------------
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

// k-th smallest card of a set (must exist)
__device__ __forceinline__ uint32_t set_select(u32x4 s, uint32_t k) {
    const uint32_t c0 = __popc(s.x), c1 = __popc(s.y), c2 = __popc(s.z);
    uint32_t w = s.x, base = 0u;
    if (k >= c0) {
        k -= c0, w = s.y, base = 32u;
        if (k >= c1) {
            k -= c1, w = s.z, base = 64u;
            if (k >= c2) k -= c2, w = s.w, base = 96u;
        }
    }
    return base + select32(w, k);
}

__device__ __forceinline__ u32x4 clear_bit(u32x4 s, uint32_t c) {
    const uint32_t bit = ~(1u << (c & 31u)), q = c >> 5;
    s.x &= (q == 0u) ? bit : ~0u;
    s.y &= (q == 1u) ? bit : ~0u;
    s.z &= (q == 2u) ? bit : ~0u;
    s.w &= (q == 3u) ? bit : ~0u;
    return s;
}

__device__ __forceinline__ u32x4 full_set(uint32_t cards) {
    u32x4 s;
    s.x = cards >= 32u ? ~0u : ((1u << cards) - 1u);
    s.y = cards >= 64u ? ~0u : cards <= 32u ? 0u : ((1u << (cards - 32u)) - 1u);
    s.z = cards >= 96u ? ~0u : cards <= 64u ? 0u : ((1u << (cards - 64u)) - 1u);
    s.w = cards >= 128u ? ~0u : cards <= 96u ? 0u : ((1u << (cards - 96u)) - 1u);
    return s;
}

__device__ __forceinline__ u32x4 hand_set(const Hand& h) {
    u32x4 s = {0u, 0u, 0u, 0u};
#pragma unroll
    for (int k = 0; k < kHand; k++) {
        const uint32_t c = hand_get(h, (uint32_t)k);
        if (c != 0xFFu) s = set_bit(s, c);
    }
    return s;
}

__device__ __forceinline__ u32x4 board_set(const Board& b) {
    const uint32_t lo[4] = {b.lo.x, b.lo.y, b.lo.z, b.lo.w};
    const uint32_t hi[4] = {b.hi.x, b.hi.y, b.hi.z, b.hi.w};
    u32x4 s = {0u, 0u, 0u, 0u};
#pragma unroll
    for (int r = 0; r < kRows; r++)
#pragma unroll
        for (int i = 0; i < 5; i++)
            if ((uint32_t)i < len_of(hi[r])) s = set_bit(s, card_at(lo[r], hi[r], i));
    return s;
}

__device__ __forceinline__ u32x4 andnot(u32x4 a, u32x4 b) { return u32x4{a.x & ~b.x, a.y & ~b.y, a.z & ~b.z, a.w & ~b.w}; }

// agents/mcts.py:62-73: at the first decision of a game (n == handsize) the
// memory is range(num_cards); every decision removes the own hand and every
// card visible on the board (cards placed and taken within one step are
// never seen -- quirk Q5, reproduced).
__device__ __forceinline__ u32x4 memorize(u32x4 mem, uint32_t n, uint32_t mcs_cards, const Hand& h, const Board& b) {
    if (n == (uint32_t)kHand) mem = full_set(mcs_cards);
    return andnot(andnot(mem, hand_set(h)), board_set(b));
}

// --------------------------------------------------------------------------
// Random word sources.  Both feed numpy's legacy masked-rejection
// random_interval; only the 32-bit word stream differs.
// --------------------------------------------------------------------------
// --------------------------------------------------------------------------
// Word buffer.  Every random_interval on this path has max <= 127 (cards
// and hand indices) and numpy masks the whole 32-bit word, so only the low
// byte of each word decides anything: the buffer keeps the low bytes of the
// next `cnt` (<= 32) words of the game's stream, byte 0 = next word.
// --------------------------------------------------------------------------
struct ByteBuf {
    uint64_t b0, b1, b2, b3;
    uint32_t cnt;

    __device__ __forceinline__ void clear() { b0 = b1 = b2 = b3 = 0ull, cnt = 0u; }

    // append k (1..8) bytes, requires cnt + k <= 32
    __device__ __forceinline__ void append(uint64_t bytes, uint32_t k) {
        bytes &= (k >= 8u) ? ~0ull : ((1ull << (8u * k)) - 1ull);
        const uint32_t bit = 8u * cnt, q = bit >> 6, off = bit & 63u;
        const uint64_t lo = bytes << off;
        const uint64_t hi = off ? (bytes >> (64u - off)) : 0ull;
        b0 |= (q == 0u) ? lo : 0ull;
        b1 |= (q == 1u) ? lo : (q == 0u) ? hi : 0ull;
        b2 |= (q == 2u) ? lo : (q == 1u) ? hi : 0ull;
        b3 |= (q == 3u) ? lo : (q == 2u) ? hi : 0ull;
        cnt += k;
    }
    // drop the next k (0..8) bytes
    __device__ __forceinline__ void drop(uint32_t k) {
        const uint32_t s = 8u * k;
        if (s >= 64u) {
            b0 = b1, b1 = b2, b2 = b3, b3 = 0ull;
        } else if (s) {
            b0 = (b0 >> s) | (b1 << (64u - s));
            b1 = (b1 >> s) | (b2 << (64u - s));
            b2 = (b2 >> s) | (b3 << (64u - s));
            b3 = b3 >> s;
        }
        cnt -= k;
    }
};

// numpy legacy random_interval(max), 1 <= max <= 127, on the buffered low
// bytes: the first of the next (up to) 8 words whose masked value is <= max
// is found with one SWAR compare, so a wave almost never loops.
// G::gen(buf) appends the next words of the stream (returns false if it
// cannot right now, see MtGen).
__device__ __forceinline__ uint64_t swar_le_mask(uint64_t x, uint32_t max) {
    // bit 7 of byte k set iff byte k of x (<= 127) is <= max (<= 127): no
    // byte borrows because (max | 0x80) - x_k lies in [1, 255]
    return ((0x0101010101010101ull * (uint64_t)(max | 0x80u)) - x) & 0x8080808080808080ull;
}

template <class G>
__device__ __forceinline__ uint32_t rng_interval(G& gen, ByteBuf& buf, uint32_t max) {
    if (max == 0u) return 0u;
    // wave-uniform top-up: all lanes with room refill together
    if (__any(buf.cnt < 8u)) gen.topup(buf);
    const uint32_t mask = 0xFFFFFFFFu >> __builtin_clz(max);
    const uint64_t mbytes = 0x0101010101010101ull * (uint64_t)mask;
    while (true) {
        if (buf.cnt == 0u) gen.force(buf);
        const uint32_t valid = min(buf.cnt, 8u);
        const uint64_t vmask = (valid >= 8u) ? ~0ull : ((1ull << (8u * valid)) - 1ull);
        const uint64_t x = buf.b0 & mbytes;
        const uint64_t t = swar_le_mask(x, max) & vmask;
        if (t) {
            const uint32_t k = (uint32_t)__builtin_ctzll(t) >> 3;
            const uint32_t v = (uint32_t)(x >> (8u * k)) & 0xFFu;
            buf.drop(k + 1u);
            return v;
        }
        buf.drop(valid);
    }
}

// K draws with the same max (DrunkHamster for every seat of one step,
// agents/random.py:9 called in seat order, play.py:38-41): the accepted
// bytes of one 16-word window are the next draws in order, so the common
// case takes all K from two SWAR compares (an 8-word window leaves some
// lane of a wave short of K accepts at most steps, and the wave then runs
// the scalar fallback for all); draws the window could not supply fall back
// to rng_interval.
__device__ __forceinline__ void buf_drop16(ByteBuf& buf, uint32_t k) {
    if (k >= 8u) {
        buf.b0 = buf.b1, buf.b1 = buf.b2, buf.b2 = buf.b3, buf.b3 = 0ull;
        buf.cnt -= 8u;
        k -= 8u;
    }
    buf.drop(k);
}

template <int K, class G>
__device__ __forceinline__ void rng_draws(G& gen, ByteBuf& buf, uint32_t max, uint32_t (&out)[K]) {
    if (max == 0u) {
#pragma unroll
        for (int k = 0; k < K; k++) out[k] = 0u;
        return;
    }
    if (__any(buf.cnt < 16u)) gen.topup(buf);
    if (__any(buf.cnt < 16u)) gen.topup(buf);
    if (buf.cnt == 0u) gen.force(buf);
    const uint32_t mask = 0xFFFFFFFFu >> __builtin_clz(max);
    const uint64_t mb = 0x0101010101010101ull * (uint64_t)mask;
    const uint32_t valid = min(buf.cnt, 16u);
    const uint32_t v0 = min(valid, 8u), v1 = valid - v0;
    const uint64_t vm0 = (v0 >= 8u) ? ~0ull : ((1ull << (8u * v0)) - 1ull);
    const uint64_t vm1 = (v1 >= 8u) ? ~0ull : ((1ull << (8u * v1)) - 1ull);
    const uint64_t x0 = buf.b0 & mb, x1 = buf.b1 & mb;
    uint64_t t0 = swar_le_mask(x0, max) & vm0, t1 = swar_le_mask(x1, max) & vm1;
    uint32_t got = 0u, last = 0u;
#pragma unroll
    for (int k = 0; k < K; k++) {
        const bool in0 = t0 != 0ull;
        const bool has = in0 || t1 != 0ull;
        const uint32_t p0 = (uint32_t)__builtin_ctzll(t0 | (1ull << 63));
        const uint32_t p1 = (uint32_t)__builtin_ctzll(t1 | (1ull << 63));
        const uint32_t pos = in0 ? p0 : 64u + p1;  // bit index (8*byte + 7) in the 16-byte window
        out[k] = (uint32_t)((in0 ? x0 : x1) >> (pos & 56u)) & 0xFFu;
        t0 = in0 ? (t0 & (t0 - 1ull)) : t0;
        t1 = in0 ? t1 : (t1 & (t1 - 1ull));
        last = has ? pos : last;
        got += has ? 1u : 0u;
    }
    // consumed: through the K-th accepted word, or the whole window
    buf_drop16(buf, got == (uint32_t)K ? (last >> 3) + 1u : valid);
#pragma unroll
    for (int k = 0; k < K; k++)
        if ((uint32_t)k >= got) out[k] = rng_interval(gen, buf, max);
}

// ---- numpy legacy MT19937, twisted lazily 8 words at a time ---------------
// State code (mt_pos[g]): bits 0..10 pos, bits 16..25 cnt.
//  Words [0,pos) of the game's 624 hold this round's values, [pos,624) the
//  previous round's (numpy's in-place twist order, done 8 words at a time
//  as draws need them; pos = 624: the round is complete).
//  cnt = words just before pos that were twisted but not consumed yet: the
//  stream continues with st[pos-cnt .. pos), then twists on.  The saved
//  state never straddles a round, so it always converts back to numpy's
//  (key, pos) form: np.random.seed(s) == init_genrand(s) with code 0, and an
//  imported numpy (key, p) is code 624 | (624 - p) << 16.
//
// A code may also straddle a round (cnt > pos): k_mt_prep twists ahead in
// place across the boundary while old-round words are still unconsumed.  The
// unconsumed old words [624 - (cnt - pos), 624) are untouched; the old
// round's words [0, pos) -- all consumed -- are recoverable from the new ones
// (the twist is invertible given the old mt[0], kept in mt0[g]), which is
// how sn_mt_get exports such a state.
//
// Round boundary.  A lane that reaches word 624 with words of the old round
// still buffered twists the new round's chunk 0 into registers but holds the
// store back ("straddle"): mt[0..8) keeps the old round's values until the
// old words are consumed (then the chunk is committed).  A launch that ends
// mid-straddle drops the held-back chunk -- it is a pure function of the old
// round and is twisted again, identically, by the next launch.
constexpr uint32_t kMtCntMask = 0x3FFu;

__device__ __forceinline__ uint32_t mt_temper(uint32_t y) {
    y ^= y >> 11;
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= y >> 18;
    return y;
}

__device__ __forceinline__ uint32_t mt_mix(uint32_t a, uint32_t b, uint32_t c) {
    const uint32_t y = (a & 0x80000000u) | (b & 0x7fffffffu);
    return c ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
}

// Inputs of one lazy refill of chunk c (8 words): mt[c..c+8), mt[c+8] and
// the run mt[j+397] (j < 227) / mt[j-227] (j >= 227), j = c..c+7.  None of
// them is written by the refills of the next 224 words.  Every loaded word
// is used: a dead lane of a vector load lets the register allocator reuse
// its register at once, which forces an s_waitcnt on the whole load.
struct MtPre {
    u32x4 a0, a1, r1;
    uint32_t a8, r00, r01, r02, r03;
};

__device__ __forceinline__ uint32_t mt_next_chunk(uint32_t c) { return (c + 8u == (uint32_t)kMtN) ? 0u : c + 8u; }

__device__ __forceinline__ MtPre mt_prefetch(const uint32_t* st, uint32_t c) {
    MtPre p;
    p.a0 = *(const u32x4*)(st + c);
    p.a1 = *(const u32x4*)(st + c + 4);
    p.a8 = st[(c + 8u == (uint32_t)kMtN) ? 0u : c + 8u];
    // the run starts at s = 1 (mod 4): s..s+2 (never past 623), s+3 (mod
    // 624, aligned), s+4..s+7 (mod 624: the chunk at 224 wraps to 1..4)
    const uint32_t s = (c < (uint32_t)(kMtN - kMtM)) ? c + kMtM : c - (uint32_t)(kMtN - kMtM);
    const uint32_t s3 = (s + 3u >= (uint32_t)kMtN) ? s + 3u - kMtN : s + 3u;
    const uint32_t s4 = (s + 4u >= (uint32_t)kMtN) ? s + 4u - kMtN : s + 4u;
    p.r00 = st[s];
    p.r01 = st[s + 1u];
    p.r02 = st[s + 2u];
    p.r03 = st[s3];
    p.r1 = u32x4{st[s4], st[s4 + 1u], st[s4 + 2u], st[s4 + 3u]};
    return p;
}

// the 8 new words of a chunk from its inputs
__device__ __forceinline__ void mt_twist8(const MtPre& p, u32x4& n0, u32x4& n1) {
    n0.x = mt_mix(p.a0.x, p.a0.y, p.r00);
    n0.y = mt_mix(p.a0.y, p.a0.z, p.r01);
    n0.z = mt_mix(p.a0.z, p.a0.w, p.r02);
    n0.w = mt_mix(p.a0.w, p.a1.x, p.r03);
    n1.x = mt_mix(p.a1.x, p.a1.y, p.r1.x);
    n1.y = mt_mix(p.a1.y, p.a1.z, p.r1.y);
    n1.z = mt_mix(p.a1.z, p.a1.w, p.r1.z);
    n1.w = mt_mix(p.a1.w, p.a8, p.r1.w);
}

// low bytes of the 8 tempered words
__device__ __forceinline__ uint64_t mt_bytes8(const u32x4& n0, const u32x4& n1) {
    const uint64_t lo = (uint64_t)((mt_temper(n0.x) & 0xFFu) | ((mt_temper(n0.y) & 0xFFu) << 8) |
                                   ((mt_temper(n0.z) & 0xFFu) << 16) | (mt_temper(n0.w) << 24));
    const uint64_t hi = (uint64_t)((mt_temper(n1.x) & 0xFFu) | ((mt_temper(n1.y) & 0xFFu) << 8) |
                                   ((mt_temper(n1.z) & 0xFFu) << 16) | (mt_temper(n1.w) << 24));
    return lo | (hi << 32);
}

// Replay of k (1..8) words that are already twisted (the unconsumed words of
// the previous launch, or an imported numpy round); scalar, out of line.
// `from` = pos - rem (mod 624): a state whose unconsumed words straddle a
// round (k_mt_prep twists ahead across it) replays the old round's tail,
// then the new round's head.
static __device__ __noinline__ uint64_t mt_replay(const uint32_t* st, uint32_t from, uint32_t k) {
    uint64_t b = 0ull;
    for (uint32_t i = 0; i < k; i++) {
        const uint32_t idx = (from + i >= (uint32_t)kMtN) ? from + i - kMtN : from + i;
        b |= (uint64_t)(mt_temper(st[idx]) & 0xFFu) << (8u * i);
    }
    return b;
}

// D = chunks (8 words) twisted per refill, 1 or 2.  A refill's loads are
// issued right after the previous refill, so D = 2 doubles the draws that
// hide their latency.  Two-chunk refills start at a multiple of 16 words
// (624 = 39 * 16, so they never cross a round); a state left at 8 mod 16 by
// a one-chunk user of the same stream realigns with one single chunk.
template <int D>
struct MtGenT {
    uint32_t* st;
    uint32_t pos, rem, straddle;
    u32x4 pn[2 * D];  // held-back first words of the next round (straddle)
    MtPre pf[D];      // inputs of the next refill's chunks

    __device__ __forceinline__ void prefetch_next() {
        const uint32_t c = (pos == (uint32_t)kMtN) ? 0u : pos;
        pf[0] = mt_prefetch(st, c);
        if (D == 2) pf[D - 1] = mt_prefetch(st, mt_next_chunk(c));
    }
    __device__ __forceinline__ void commit() {
#pragma unroll
        for (int k = 0; k < 2 * D; k++) *(u32x4*)(st + 4 * k) = pn[k];
        straddle = 0u;
    }
    // keep = true: continue after bytes already in buf (RingGen's fallback)
    __device__ __forceinline__ void load(uint32_t* state, uint32_t code, ByteBuf& buf, bool keep = false) {
        st = state;
        pos = code & 0x7FFu;
        rem = (code >> 16) & kMtCntMask;
        straddle = 0u;
        if (!keep) buf.clear();
        prefetch_next();
    }
    // state code for mt_pos[]; commits or drops a held-back chunk
    __device__ __forceinline__ uint32_t save(const ByteBuf& buf) {
        if (straddle) {
            if (buf.cnt > 8u * D) return (uint32_t)kMtN | ((buf.cnt - 8u * D) << 16);  // old words left: drop
            commit();
            return 8u * D | (buf.cnt << 16);
        }
        return pos | ((rem + buf.cnt) << 16);
    }
    // one batch of words; false if it cannot run now (a straddle whose old
    // words are still buffered)
    __device__ __forceinline__ bool gen(ByteBuf& buf);
    __device__ __forceinline__ void topup(ByteBuf& buf) {
        if (buf.cnt <= 32u - 8u * D) gen(buf);
    }
    __device__ __forceinline__ void force(ByteBuf& buf) { gen(buf); }  // cnt == 0: always succeeds
};

template <int D>
__device__ __forceinline__ bool MtGenT<D>::gen(ByteBuf& buf) {
    if (rem) {
        const uint32_t k = min(8u, rem);
        buf.append(mt_replay(st, (pos >= rem) ? pos - rem : pos + kMtN - rem, k), k);
        rem -= k;
        return true;
    }
    if (straddle) {
        if (buf.cnt > 8u * D) return false;
        commit();  // old round consumed
    }
    const bool wrap = (pos == (uint32_t)kMtN);
    const uint32_t i = wrap ? 0u : pos;
    const bool two = (D == 2) && !(i & 8u);
    u32x4 n[4];
    mt_twist8(pf[0], n[0], n[1]);
    n[2] = n[3] = u32x4{0u, 0u, 0u, 0u};
    if (D == 2) mt_twist8(pf[D - 1], n[2], n[3]);
    if (wrap && buf.cnt) {
#pragma unroll
        for (int k = 0; k < 2 * D; k++) pn[k] = n[k];
        straddle = 1u;
    } else {
        *(u32x4*)(st + i) = n[0];
        *(u32x4*)(st + i + 4) = n[1];
        if (two) {
            *(u32x4*)(st + i + 8) = n[2];
            *(u32x4*)(st + i + 12) = n[3];
        }
    }
    buf.append(mt_bytes8(n[0], n[1]), 8u);
    if (two) buf.append(mt_bytes8(n[2], n[3]), 8u);
    pos = i + (two ? 16u : 8u);
    // Keep the next loads below the last use of the inputs just consumed:
    // hoisted above it, they get fresh registers and the loop's phi copies
    // them back at once -- an s_waitcnt right behind the loads that made the
    // prefetch worthless (seen in the gfx950 ISA).
    asm volatile("" ::"v"(n[0].x), "v"(n[1].w), "v"(n[2].x), "v"(n[3].w) : "memory");
    prefetch_next();
    return true;
}

using MtGen = MtGenT<1>;

// numpy (key, pos) form of a state code, host and device: the caller has
// finished the round in place when pos < 624 (mt_finish_round)
// (a straddling code, cnt > pos, is in the previous round: its numpy key is
// that round, restored by the caller -- sn_mt_get)
__host__ __device__ __forceinline__ int mt_numpy_pos(uint32_t code) {
    const uint32_t p = code & 0x7FFu, cnt = (code >> 16) & kMtCntMask;
    if (p == 0u) return kMtN;  // previous round complete, next draw twists
    return (cnt > p) ? (int)(kMtN + p - cnt) : (int)(p - cnt);
}
__host__ __device__ __forceinline__ uint32_t mt_code_from_numpy(int pos) {
    return (pos >= kMtN) ? 0u : ((uint32_t)kMtN | ((uint32_t)(kMtN - pos) << 16));
}

// ---- Philox4x32-10 counter-based stream -----------------------------------
// word w of game s = philox({w/4 lo, w/4 hi, s lo, s hi}, seed)[w % 4]
__device__ __forceinline__ u32x4 philox4x32_10(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0,
                                               uint32_t k1) {
#pragma unroll
    for (int r = 0; r < 10; r++) {
        const uint32_t lo0 = 0xD2511F53u * c0, hi0 = __umulhi(0xD2511F53u, c0);
        const uint32_t lo1 = 0xCD9E8D57u * c2, hi1 = __umulhi(0xCD9E8D57u, c2);
        const uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
        c0 = n0, c1 = lo1, c2 = n2, c3 = lo0;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    u32x4 o;
    o.x = c0, o.y = c1, o.z = c2, o.w = c3;
    return o;
}

struct PhiloxGen {
    uint32_t k0, k1, s0, s1;
    uint64_t next_blk;  // next block to generate (words 4*next_blk ..)

    __device__ __forceinline__ uint64_t block_bytes(uint64_t blk) const {
        const u32x4 o = philox4x32_10((uint32_t)blk, (uint32_t)(blk >> 32), s0, s1, k0, k1);
        return (uint64_t)((o.x & 0xFFu) | ((o.y & 0xFFu) << 8) | ((o.z & 0xFFu) << 16) | (o.w << 24));
    }
    __device__ __forceinline__ void load(uint32_t seed_lo, uint32_t seed_hi, uint64_t gid, uint64_t consumed,
                                         ByteBuf& buf) {
        k0 = seed_lo, k1 = seed_hi;
        s0 = (uint32_t)gid, s1 = (uint32_t)(gid >> 32);
        buf.clear();
        next_blk = consumed >> 2;
        const uint32_t j = (uint32_t)consumed & 3u;
        if (j) {  // resume inside a block
            buf.append(block_bytes(next_blk), 4u);
            next_blk++;
            buf.drop(j);
        }
    }
    __device__ __forceinline__ uint64_t consumed(const ByteBuf& buf) const { return 4ull * next_blk - buf.cnt; }
    __device__ __forceinline__ void gen8(ByteBuf& buf) {
        const uint64_t a = block_bytes(next_blk), b = block_bytes(next_blk + 1);
        buf.append(a | (b << 32), 8u);
        next_blk += 2;
    }
    __device__ __forceinline__ void topup(ByteBuf& buf) {
        if (buf.cnt <= 24u) gen8(buf);
    }
    __device__ __forceinline__ void force(ByteBuf& buf) { gen8(buf); }
};

// a 24-bit uniform in [0, 1) from word 0 of one Philox block
__device__ __forceinline__ float philox_uniform(uint32_t k0, uint32_t k1, uint64_t stream, uint32_t counter) {
    const u32x4 o = philox4x32_10(counter, 0u, (uint32_t)stream, (uint32_t)(stream >> 32), k0, k1);
    return (float)(o.x >> 8) * (1.0f / 16777216.0f);
}

}  // namespace sechs

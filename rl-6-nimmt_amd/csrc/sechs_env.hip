// sechs_env.hip -- vectorised SechsNimmtEnv for gfx950 + the C ABI (include/sechs.h).
//
// Device state layout: sechs_state.h.
// A launch loads each game into VGPRs, plays `steps` env-steps and stores it
// back; per step the only HBM traffic is the caller's outputs and, in
// numpy-compat mode, the MT19937 words (8 per refill, 16-B accesses).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <string>
#include <type_traits>

#define SECHS_DEBUG_HERE  // SN_DASSERT is live in this file's kernels (libsechs_debug.so only)
#include "sechs_state.h"

using namespace sechs;

// ============================================================================
// kernels
// ============================================================================
__global__ void k_seed(DevState s) {
    const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= s.B) return;
    if (s.rng_mode == RNG_NUMPY_MT) {
        // np.random.seed(seed + gid): init_genrand; numpy pos 624 == lazy code 0
        uint32_t* st = s.mt + g * kMtN;
        uint32_t v = (uint32_t)(s.seed + s.game_offset + (uint64_t)g);
        st[0] = v;
        for (int i = 1; i < kMtN; i++) {
            v = 1812433253u * (v ^ (v >> 30)) + (uint32_t)i;
            st[i] = v;
        }
        s.mt_pos[g] = 0u;
    } else {
        s.ctr[g] = 0u;
    }
    for (int p = 0; p < s.N; p++) s.sum_res[(int64_t)p * s.B + g] = 0;
    s.episodes[g] = 0;
}

template <int N, int MODE, bool LG = false>
__global__ __launch_bounds__(kBlock) void k_reset(DevState s, const uint8_t* decks) {
    __shared__ uint8_t lds_deck[kBlock * kDealStride];
    const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= s.B) return;
    Game<N> G;
    if (decks) {
        const uint8_t* d = decks + g * s.C;
        deal_from<N>([&](int i) -> uint32_t { return d[i]; }, s.C, G);
    } else {
        typename RngOf<MODE>::T rng;
        ByteBuf buf;
        RngOf<MODE>::load(s, g, rng, buf);
        uint32_t lg = 0u;
        if (LG) lg = league_draw(rng, buf, s.lg_K, s.lg_lo, s.lg_hi);  // Tournament.play_game: seats, then the deal
        uint8_t* slot = lds_deck + threadIdx.x * kDealStride;
        deck_shuffle2(rng, buf, slot, s.C);
        deal_from_deck<N>(slot, s.C, G);
        if (LG) {
#pragma unroll
            for (int p = 0; p < N; p++)
                if ((uint32_t)p >= (lg & 15u)) G.hand[p].lo = ~0ull, G.hand[p].hi = ~0u;
            s.lgs[g] = lg;
        }
        RngOf<MODE>::store(s, g, rng, buf);
    }
    store_game<N>(s, g, G);
}

template <int N>
__global__ __launch_bounds__(kBlock) void k_reset_to(DevState s, const int8_t* board, const int8_t* hands) {
    const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= s.B) return;
    Game<N> G;
#pragma unroll
    for (int p = 0; p < N; p++) {
        u32x4 set = {0u, 0u, 0u, 0u};
        for (int k = 0; k < kHand; k++) {
            const int c = hands[(g * N + p) * kHand + k];
            if (c >= 0) set = set_bit(set, (uint32_t)c);
        }
        G.hand[p] = hand_from_set(set);
        G.score[p] = 0;
    }
    uint32_t lo[4], hi[4];
#pragma unroll
    for (int r = 0; r < kRows; r++) {
        uint32_t l = 0, card4 = 0, len = 0, heads = 0, end = 0;
        for (int i = 0; i < kThreshold; i++) {
            const int c = board[(g * kRows + r) * kThreshold + i];
            if (c < 0) continue;
            if (len < 4) l |= (uint32_t)c << (8 * len);
            else card4 = (uint32_t)c;
            heads += heads_of((uint32_t)c);
            end = (uint32_t)c;
            len++;
        }
        lo[r] = l;
        hi[r] = (card4 & 0xFFu) | (len << 8) | (heads << 16) | (end << 24);
    }
    G.b.lo = u32x4{lo[0], lo[1], lo[2], lo[3]};
    G.b.hi = u32x4{hi[0], hi[1], hi[2], hi[3]};
    store_game<N>(s, g, G);
}

// numpy-MT twist-ahead for a k_play launch: one wave per game twists, in
// place and 64 consecutive words per instruction (every load and store one
// contiguous run), the game's stream far enough that ring_w words lie
// twisted and unconsumed, and writes their tempered low bytes to the ring
// (RingGen).  numpy's in-place twist order makes any 227 consecutive words
// independent: word i reads mt[i], mt[i+1] (both still the previous round's)
// and mt[i+397] (previous round, i < 227) or mt[i-227] (this round, twisted
// 227 words earlier).  So the words this launch twists first (j < 227) have
// every input in memory already: all their loads are issued before any
// store (the wave keeps 3 * (NB + 1) loads in flight), and only words j >=
// 227 (a nearly empty ring, or 512-word rings) wait for those stores.  The
// twist pointer stays a multiple of 8 (MtGen's chunking).  Twisting word 0
// of a new round while old words are unconsumed makes the code straddle;
// the overwritten old mt[0] goes to mt0[g] so sn_mt_get can still export
// numpy's key.
constexpr int kPrepGamesPerWave = 4;

template <int NB, int GPW>  // ring_w / 64, games per wave
__global__ __launch_bounds__(kBlock) void k_mt_prep(DevState s) {
    constexpr uint32_t W = 64u * NB;
    constexpr uint32_t D = kMtN - kMtM;  // 227
    const int64_t g0 = ((int64_t)blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6)) * GPW;
    if (g0 >= s.B) return;  // whole waves
    const uint32_t lane = threadIdx.x & 63u;
    uint32_t rem[GPW], KT[GPW], T0[GPW], base[GPW];
    uint32_t A[GPW][NB + 1], C[GPW][NB + 1];
    // Word k of game q (k = 0 .. KT) sits at twist index base + k (mod 624):
    // the first rem are twisted and unconsumed (re-tempered into the ring),
    // the rest are twisted now.  All loads of all GPW games go out first.
    // one load for the GPW state codes (lane q holds game g0 + q's): a
    // per-game load here would make each game's wait drain the previous
    // game's loads (vmcnt counts in order)
    const uint32_t codes = (lane < (uint32_t)GPW) ? s.mt_pos[min(g0 + (int64_t)lane, s.B - 1)] : 0u;
#pragma unroll
    for (int q = 0; q < GPW; q++) {
        const int64_t g = min(g0 + q, s.B - 1);  // a short last wave repeats its last game (loads only)
        const uint32_t code = __builtin_amdgcn_readlane(codes, q);
        const uint32_t T = code & 0x7FFu;
        rem[q] = (code >> 16) & kMtCntMask;
        const uint32_t add = (rem[q] >= W) ? 0u : ((W - rem[q] + 7u) & ~7u);
        KT[q] = rem[q] + add;
        T0[q] = (T == (uint32_t)kMtN) ? 0u : T;
        base[q] = T0[q] + kMtN - rem[q];  // + k, mod 624
        const uint32_t* st = s.mt + g * kMtN;
#pragma unroll
        for (int b = 0; b <= NB; b++) {
            const uint32_t k = 64u * b + lane;
            uint32_t idx = base[q] + k;
            idx = (idx >= (uint32_t)kMtN) ? idx - kMtN : idx;
            idx = (idx >= (uint32_t)kMtN) ? idx - kMtN : idx;
            if (k <= KT[q]) A[q][b] = st[idx];
            if (k >= rem[q] && k < KT[q] && k - rem[q] < D) C[q][b] = st[(idx < D) ? idx + kMtM : idx - D];
        }
    }
    uint32_t* ring = (uint32_t*)s.ring;
#pragma unroll
    for (int q = 0; q < GPW; q++) {
        const int64_t g = g0 + q;
        if (g >= s.B) break;
        uint32_t* st = s.mt + g * kMtN;
        const uint32_t r = rem[q], kt = KT[q];
#pragma unroll
        for (int b = 0; b <= NB; b++) {
            if (b == NB && kt <= W) break;
            const uint32_t k = 64u * b + lane;
            uint32_t idx = base[q] + k;
            idx = (idx >= (uint32_t)kMtN) ? idx - kMtN : idx;
            idx = (idx >= (uint32_t)kMtN) ? idx - kMtN : idx;
            // mt[idx + 1] = word k + 1 = the next lane's A (lane 63: lane 0 of the next batch)
            const uint32_t nxt = (b < NB) ? __shfl(A[q][b < NB ? b + 1 : b], 0) : 0u;
            uint32_t bb = __shfl_down(A[q][b], 1);
            bb = (lane == 63u) ? nxt : bb;
            uint32_t v = A[q][b];
            if (k >= r && k < kt && k - r < D) {
                v = mt_mix(A[q][b], bb, C[q][b]);
                st[idx] = v;
                if (idx == 0u) s.mt0[g] = A[q][b];
            }
            if (b < NB) {  // ring bytes: 4 words per dword (lanes 4m..4m+3)
                const uint32_t y = mt_temper(v) & 0xFFu;
                const uint32_t d = y | (__shfl_down(y, 1) << 8) | (__shfl_down(y, 2) << 16) | (__shfl_down(y, 3) << 24);
                if ((lane & 3u) == 0u) ring[(((int64_t)(k >> 4)) * s.B + g) * 4 + ((k >> 2) & 3u)] = d;
            }
        }
        // words j >= 227 read words twisted just above: in order, after those stores
        if (kt > r + D) {
            for (uint32_t k0 = ((r + D) & ~63u); k0 < kt; k0 += 64u) {
                const uint32_t k = k0 + lane;
                uint32_t v = 0u;
                if (k >= r + D && k < kt) {
                    uint32_t idx = base[q] + k;
                    idx = (idx >= (uint32_t)kMtN) ? idx - kMtN : idx;
                    idx = (idx >= (uint32_t)kMtN) ? idx - kMtN : idx;
                    const uint32_t a = st[idx];
                    v = mt_mix(a, st[(idx + 1u == (uint32_t)kMtN) ? 0u : idx + 1u], st[(idx < D) ? idx + kMtM : idx - D]);
                    st[idx] = v;
                    if (idx == 0u) s.mt0[g] = a;
                }
                const uint32_t y = mt_temper(v) & 0xFFu;
                const uint32_t d = y | (__shfl_down(y, 1) << 8) | (__shfl_down(y, 2) << 16) | (__shfl_down(y, 3) << 24);
                if ((lane & 3u) == 0u && k < W && k + 3u >= r + D) {
                    uint32_t* dst = ring + (((int64_t)(k >> 4)) * s.B + g) * 4 + ((k >> 2) & 3u);
                    if (k >= r + D) {
                        *dst = d;
                    } else {  // dword shared with words stored above: merge the new bytes
                        const uint32_t keep = (1u << (8u * (r + D - k))) - 1u;
                        *dst = (*dst & keep) | (d & ~keep);
                    }
                }
            }
        }
        if (lane == 0u && kt > r) {
            const uint32_t Tn = T0[q] + (kt - r);
            s.mt_pos[g] = ((Tn > (uint32_t)kMtN) ? Tn - kMtN : Tn) | (kt << 16);
        }
    }
}

// ============================================================================
// Pipelined numpy-MT twist-ahead (SN_OPT_PIPELINE, the default for numpy-mode
// DrunkHamster rollouts).  k_mt_ahead keeps each game's stream twisted
// kPipeLead words past the consumer position of the play launch before last,
// writing the tempered low bytes into a per-game circular ring indexed by
// absolute stream position (pring).  It reads only state no running kernel
// writes (pabsc of the launch before last, its own ptend / ptp), and the
// ring slots it fills are never the ones the running k_play reads (lead +
// one launch < kPipeRing), so it runs on a side stream CONCURRENTLY with
// k_play (launch i+1's twist beside launch i's game loop: memory-bound work
// beside latency-bound work, on the same CUs).  One wave per game; 64
// consecutive words per instruction; the first 224 words have all inputs in
// memory (loads first), later ones follow in order (word j reads j - 227).
// INIT: start from the MtGen state code (re-temper its twisted-unconsumed
// words into the ring first).
// ============================================================================
#ifndef SECHS_NT_OBS
#define SECHS_NT_OBS 1
#endif
#ifndef SECHS_NT_MORE
#define SECHS_NT_MORE 1
#endif
// streaming (non-temporal) stores for what no later kernel finds in L2
// anyway (the 155 MB of trajectory outputs and the MT words / ring bytes a
// launch writes): measured 5.77 -> 6.4 G env-steps/s.  Non-temporal LOADS
// of the MT state were measured slower (5.5 G/s: consecutive lanes share
// lines through L2), so loads stay normal.
template <class T>
__device__ __forceinline__ void st_nt(T* p, T v, bool nt) {
    if (nt) __builtin_nontemporal_store(v, p);
    else *p = v;
}

struct AheadArgs {
    int cin;   // pabsc parity holding the consumer position to lead (INIT: written)
    int tin;   // ptend parity of the previous prep (steady)
    int tout;  // ptend parity written
    int lead;  // words to keep twisted past the consumer (kPipeLead; smaller only to test the overrun path)
    uint32_t* perr_mirror;  // host-mapped copy of *perr, refreshed at launch start (off the play stream)
    int cin_copy;  // INIT: also write the start position to this pabsc slot (-1: none; decode-ahead: the play slot)
};

// One whole MT19937 round of game G, twisted by the whole wave in LDS (w:
// 624 words; k_mt_ahead's whole-round twists), its
// tempered low bytes to the ring at stream positions te .. te + 623 (te is
// 8-aligned: rounds are 624 = 78 x 8 words).  numpy's in-place order in
// three dependency-free phases: words 0..226 read old words only (mt[i+1],
// mt[i+397]); 227..453 read old mt[i+1] and the new mt[i-227] of phase 1;
// 454..623 the new mt[i-227] of phase 2 (and mt[623] the new mt[0]).  One
// HBM read and one write per word (k_mt_ahead's partial twists read the
// i+397 input a second time).  Returns the old mt[0] (the one word the
// sync-time untwist cannot recover, mt0).
// v: the round's old words (word 64k + lane in v[k]), loaded by the caller
// (a round ahead: mt_round_load)
__device__ __forceinline__ void mt_round_load(const DevState& s, int64_t G, uint32_t lane, uint32_t (&v)[10]) {
    const uint32_t* st = s.mt + G * kMtN;
#pragma unroll
    for (int k = 0; k < 10; k++) {
        const uint32_t i = 64u * k + lane;
        v[k] = (i < (uint32_t)kMtN) ? st[i] : 0u;
    }
}

__device__ __forceinline__ void mt_round_to_lds(uint32_t lane, uint32_t* w, const uint32_t (&v)[10]) {
#pragma unroll
    for (int k = 0; k < 10; k++) {
        const uint32_t i = 64u * k + lane;
        if (i < (uint32_t)kMtN) w[i] = v[k];
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
}

// w holds the round's old words (mt_round_to_lds)
__device__ __forceinline__ uint32_t mt_twist_round(const DevState& s, int64_t G, uint32_t lane, uint32_t* w,
                                                     uint32_t te) {
    constexpr uint32_t D = kMtN - kMtM;  // 227
    uint32_t* st = s.mt + G * kMtN;
    const uint32_t old0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)w[0]);
    uint32_t nv[4];
#pragma unroll
    for (int k = 0; k < 4; k++) {  // phase 1: i < 227
        const uint32_t i = 64u * k + lane;
        nv[k] = (i < D) ? mt_mix(w[i], w[i + 1u], w[i + kMtM]) : 0u;
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const uint32_t i = 64u * k + lane;
        if (i < D) w[i] = nv[k];
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
#pragma unroll
    for (int k = 0; k < 4; k++) {  // phase 2: 227 <= i < 454
        const uint32_t i = D + 64u * k + lane;
        nv[k] = (i < 2u * D) ? mt_mix(w[i], w[i + 1u], w[i - D]) : 0u;
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const uint32_t i = D + 64u * k + lane;
        if (i < 2u * D) w[i] = nv[k];
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
#pragma unroll
    for (int k = 0; k < 3; k++) {  // phase 3: 454 <= i < 624
        const uint32_t i = 2u * D + 64u * k + lane;
        nv[k] = (i < (uint32_t)kMtN) ? mt_mix(w[i], w[(i + 1u == (uint32_t)kMtN) ? 0u : i + 1u], w[i - D]) : 0u;
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
#pragma unroll
    for (int k = 0; k < 3; k++) {
        const uint32_t i = 2u * D + 64u * k + lane;
        if (i < (uint32_t)kMtN) w[i] = nv[k];
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    // the new round to HBM (state words), its tempered low bytes to the ring
    // (4 per dword: dword d holds stream positions te + 4d .. te + 4d + 3)
#pragma unroll
    for (int k = 0; k < 10; k++) {
        const uint32_t i = 64u * k + lane;
        if (i < (uint32_t)kMtN) st_nt(&st[i], w[i], SECHS_NT_MORE);
    }
    uint8_t* ring = (uint8_t*)s.pring;
#pragma unroll
    for (int k = 0; k < 3; k++) {
        const uint32_t d = 64u * k + lane;
        if (d < (uint32_t)kMtN / 4u) {
            const u32x4 x = *(const u32x4*)(w + 4u * d);
            const uint32_t y = (mt_temper(x.x) & 0xFFu) | ((mt_temper(x.y) & 0xFFu) << 8) |
                               ((mt_temper(x.z) & 0xFFu) << 16) | ((mt_temper(x.w) & 0xFFu) << 24);
            const uint32_t ri = (te + 4u * d) & (uint32_t)(kPipeRing - 1);
            st_nt((uint32_t*)(ring + ring_byte(ri, G, s.B)), y, SECHS_NT_MORE);  // ri is 4-aligned
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");  // the LDS reads before the area's next use
    return old0;
}

// ROUND (SN_OPT_TWIST_ROUND): twist whole MT rounds instead of exactly the
// words the lead needs.  A twist that is due first completes the current
// round (the per-64-word form below), then -- if the lead is still short --
// twists the next round of 624 words in LDS: the round's old words are read
// once, every input of numpy's in-place order (mt[i+1], mt[i+397] / the new
// mt[i-227]) comes from LDS, and each new word is written once: 8 B of MT
// traffic per word instead of 12 (the X input of a partial twist is a
// second HBM read).  The lead then ranges up to 600 + 624 words, so the
// ring holds kPipeRing = 2048 bytes per game; a handle synchronised while
// the array is a round ahead of its consumer is untwisted (k_pipe_code).
template <bool INIT, bool ROUND = false>
__global__ __launch_bounds__(kBlock) void k_mt_ahead(DevState s, AheadArgs a) {
    constexpr uint32_t D = kMtN - kMtM;  // 227
    constexpr uint32_t P1 = 224;          // words twisted before any store (all inputs already in memory)
    const int64_t g = (int64_t)blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6);
    if (g >= s.B) return;  // whole waves
    const uint32_t lane = threadIdx.x & 63u;
    const int64_t B = s.B;
    // publish the overrun count so far (every k_play before the running one)
    // to the host without a sync; sn_rollout reads it at entry
    if (g == 0 && lane == 0u && a.perr_mirror)
        __hip_atomic_store(a.perr_mirror, __hip_atomic_load(s.perr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    uint32_t* st = s.mt + g * kMtN;
    uint8_t* ring = (uint8_t*)s.pring;
    uint32_t Tp, t0, c;
    if (INIT) {
        const uint32_t code = s.mt_pos[g];
        Tp = code & 0x7FFu;
        const uint32_t rem = (code >> 16) & kMtCntMask;
        t0 = 0u;
        c = 0u - rem;
        for (uint32_t k0 = 0; k0 < rem; k0 += 64u) {  // twisted, unconsumed: stream index Tp - rem + k (mod 624)
            const uint32_t k = k0 + lane;
            if (k < rem) {
                const uint32_t v = st[(Tp + kMtN - rem + k) % (uint32_t)kMtN];
                const uint32_t ri = (c + k) & (uint32_t)(kPipeRing - 1);
                ring[ring_byte(ri, g, B)] = (uint8_t)(mt_temper(v) & 0xFFu);
            }
        }
        if (lane == 0u) {
            s.pabsc[(int64_t)a.cin * B + g] = c;
            if (a.cin_copy >= 0) s.pabsc[(int64_t)a.cin_copy * B + g] = c;
        }
    } else {
        Tp = s.ptp[g];
        t0 = s.ptend[(int64_t)a.tin * B + g];
        c = s.pabsc[(int64_t)a.cin * B + g];
    }
    // signed: a consumer past the twisted end means a play lane overran
    // (counted there too); twist nothing rather than underflow the lead
    const int32_t lead = (int32_t)(t0 - c);
    if (lead < 0 && lane == 0u) atomicAdd(s.perr, 1u);
    const uint32_t T0 = (Tp == (uint32_t)kMtN) ? 0u : Tp;
    // ROUND: the words completing the current round (none at a round boundary)
    const uint32_t n = ROUND ? ((lead >= 0 && lead < a.lead && T0 != 0u) ? (uint32_t)kMtN - T0 : 0u)
                             : ((lead >= 0 && lead < a.lead) ? (((uint32_t)(a.lead - lead)) & ~7u) : 0u);
    auto ring_dword = [&](uint32_t j, uint32_t v) {  // t0 is 8-aligned: lanes 4m..4m+3 share one dword
        const uint32_t y = mt_temper(v) & 0xFFu;
        const uint32_t d = y | (__shfl_down(y, 1) << 8) | (__shfl_down(y, 2) << 16) | (__shfl_down(y, 3) << 24);
        const uint32_t ri = (t0 + j) & (uint32_t)(kPipeRing - 1);
        if ((lane & 3u) == 0u && j < n) st_nt((uint32_t*)(ring + ring_byte(ri, g, B)), d, SECHS_NT_MORE);  // ri 4-aligned
    };
    // Word-0 crossings of this launch (wave-uniform count): the overwritten
    // old mt[0] of each.  k_pipe_code's untwist needs one per round the array
    // runs ahead of the consumer -- up to three with SN_OPT_TWIST_EVERY = 3
    // (a lead of 1 800 words) -- so mt0[k B + g] keeps the k-th newest; kept
    // in registers here, so no load follows a store of this launch.
    uint32_t ncross = 0u, old0[kMt0Levels] = {};
    auto cross = [&](bool hit, uint32_t old) {
        const uint64_t m = __ballot(hit);
        if (m) {
            const uint32_t v = __shfl(old, (int)__builtin_ctzll(m));
#pragma unroll
            for (int k = kMt0Levels - 1; k > 0; k--) old0[k] = old0[k - 1];  // newest first
            old0[0] = v;
            ncross++;
        }
    };
    // phase 1: words 0 .. min(n, 224)
    uint32_t A[4] = {0u, 0u, 0u, 0u}, Bv[4], Cv[4], IX[4];
#pragma unroll
    for (int b = 0; b < 4; b++) {
        const uint32_t j = 64u * b + lane;
        IX[b] = 0xFFFFu;
        if (j < n && j < P1) {
            const uint32_t idx = (T0 + j) % (uint32_t)kMtN;
            IX[b] = idx;
            A[b] = st[idx];
            Bv[b] = st[(idx + 1u == (uint32_t)kMtN) ? 0u : idx + 1u];
            Cv[b] = st[(idx < D) ? idx + kMtM : idx - D];
        }
    }
#pragma unroll
    for (int b = 0; b < 4; b++) {
        if (64u * b >= min(n, P1)) break;
        const uint32_t j = 64u * b + lane;
        uint32_t v = 0u;
        if (IX[b] != 0xFFFFu) {
            v = mt_mix(A[b], Bv[b], Cv[b]);
            st_nt(&st[IX[b]], v, SECHS_NT_MORE);
        }
        cross(IX[b] == 0u, A[b]);
        ring_dword(j, v);
    }
    // phase 2: words 224 .. n, in order (their inputs include words just twisted)
    for (uint32_t j0 = P1; j0 < n; j0 += 64u) {
        const uint32_t j = j0 + lane;
        uint32_t v = 0u, aa = 0u;
        bool at0 = false;
        if (j < n) {
            const uint32_t idx = (T0 + j) % (uint32_t)kMtN;
            aa = st[idx];
            v = mt_mix(aa, st[(idx + 1u == (uint32_t)kMtN) ? 0u : idx + 1u], st[(idx < D) ? idx + kMtM : idx - D]);
            st[idx] = v;
            at0 = idx == 0u;
        }
        cross(at0, aa);
        ring_dword(j, v);
    }
    uint32_t Tn = Tp, te = t0 + n;
    if (n) {
        Tn = T0 + n;
        while (Tn > (uint32_t)kMtN) Tn -= kMtN;
    }
    if constexpr (ROUND) {
        // whole rounds in LDS while the lead is short (one per twist at K <= 2, up to kMt0Levels - 1)
        for (int rr = 0; rr < kMt0Levels - 1 && lead >= 0 && lead + (int32_t)(te - t0) < a.lead; rr++) {
            __shared__ __attribute__((aligned(16))) uint32_t wround[kBlock / 64][kMtN];
            uint32_t* w = wround[threadIdx.x >> 6];
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");  // the words twisted before: stored first
            uint32_t v[10];
            mt_round_load(s, g, lane, v);  // all ten loads in flight at once
            mt_round_to_lds(lane, w, v);
            // three dependency-free phases (mt_twist_round); old mt[0]: the one word the untwist cannot recover
            cross(true, mt_twist_round(s, g, lane, w, te));
            te += kMtN;
            Tn = kMtN;
        }
    }
    SN_DASSERT(ncross <= (uint32_t)kMt0Levels);
    if (lane == 0u) {
        s.ptp[g] = Tn;
        s.ptend[(int64_t)a.tout * B + g] = te;
        if (ncross) {  // the stack of crossings, newest first: this launch's, then the older ones
            uint32_t stk[kMt0Levels];
            for (int k = 0; k < kMt0Levels; k++) stk[k] = s.mt0[k * B + g];
            for (int k = 0; k < kMt0Levels; k++)
                s.mt0[k * B + g] = (k < (int)ncross) ? old0[k] : stk[k - (int)ncross];
        }
    }
}

// state code of a pipelined handle (for MtGen users and sn_mt_get):
// twist pointer | (twisted end - consumer) << 16
__device__ __forceinline__ uint32_t mt_untwist_y_dev(uint32_t t) {
    const uint32_t lsb = t >> 31;  // the twist constant's top bit is set, y >> 1's is not
    return (((lsb ? (t ^ 0x9908b0dfu) : t)) << 1) | lsb;
}

__global__ __launch_bounds__(kBlock) void k_pipe_code(DevState s, int cin, int tin) {
    const int64_t g = (int64_t)blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6);  // one wave per game
    if (g >= s.B) return;  // whole waves
    const uint32_t lane = threadIdx.x & 63u;
    int32_t rem = (int32_t)(s.ptend[(int64_t)tin * s.B + g] - s.pabsc[(int64_t)cin * s.B + g]);
    if (rem < 0 && lane == 0u) atomicAdd(s.perr, 1u);  // an overrun (already counted): the stream is lost
    uint32_t tp = s.ptp[g];
    // The array ran ahead of the consumer's round (whole-round twists, or
    // the K-group lead of SN_OPT_TWIST_EVERY): undo its newest round's
    // twisted words [0, tp) in place (new -> old), the host mt_unstraddle,
    // until the unconsumed words fit one array.  With y[j] the twist's
    // intermediate (top(old[j]) | low(old[j+1])): y[j] = U(new[j] ^ X[j]),
    // X[j] = new[j-227] for j >= 227 -- all from new words, in parallel --
    // and old[j+397] for j < 227, whose y[j+396], y[j+397] the first phase
    // gave (or the word was never twisted: j + 397 >= tp); then old[j] =
    // top(y[j]) | low(y[j-1]), old[0]'s low half from mt0 (newest crossing
    // first, then the ones before).  One wave per game, in LDS.
    __shared__ uint32_t sw[kBlock / 64][kMtN], sy[kBlock / 64][kMtN];
    uint32_t* w = sw[threadIdx.x >> 6];
    uint32_t* y = sy[threadIdx.x >> 6];
    uint32_t* a = s.mt + g * kMtN;
    constexpr uint32_t D = kMtN - kMtM;
    int lvl = 0;
    if (rem > kMtN) {
        for (uint32_t j = lane; j < (uint32_t)kMtN; j += 64u) w[j] = a[j];
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    }
    for (; rem > kMtN && lvl < kMt0Levels; lvl++) {
        SN_DASSERT(tp >= 1u && tp <= (uint32_t)kMtN);
        if (tp < 1u || tp > (uint32_t)kMtN) break;
        for (uint32_t j = D + lane; j < tp; j += 64u) y[j] = mt_untwist_y_dev(w[j] ^ w[j - D]);
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        for (uint32_t j = lane; j < min(D, tp); j += 64u) {
            const uint32_t k = j + kMtM;  // 397 .. 623
            const uint32_t old_k = (k < tp) ? ((y[k] & 0x80000000u) | (y[k - 1u] & 0x7fffffffu)) : w[k];
            y[j] = mt_untwist_y_dev(w[j] ^ old_k);
        }
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        const uint32_t m0 = s.mt0[lvl * s.B + g];
        for (uint32_t j = lane; j < tp; j += 64u)
            w[j] = (y[j] & 0x80000000u) | ((j ? y[j - 1u] : m0) & 0x7fffffffu);
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        rem -= (int32_t)tp;
        tp = kMtN;
    }
    if (lvl) {
        for (uint32_t j = lane; j < (uint32_t)kMtN; j += 64u) a[j] = w[j];
        if (lane == 0u)
            for (int k = 0; k < kMt0Levels; k++)  // the crossings not undone are the newest now
                s.mt0[k * s.B + g] = (k + lvl < kMt0Levels) ? s.mt0[(k + lvl) * s.B + g] : 0u;
    }
    SN_DASSERT(rem <= kMtN);
    if (lane == 0u) s.mt_pos[g] = tp | ((uint32_t)max(rem, 0) << 16);
}

// ---- k_play phase profiler (diagnostics; built only with -DSECHS_PHASE_PROF,
// the libsechs_prof.so variant).  Each wave accumulates shader-clock cycles
// per phase of its step loop and adds them to g_phase at exit; the clock
// reads add lgkmcnt waits at the phase marks, so the split is indicative.
// PH_B1 / PH_B2: a k_play_split play wave waiting at its barriers; PR_*: the
// producer waves' phases.  g_phase[PH_N] counts play waves, [PH_N + 1] producers.
enum {
    PH_PROLOGUE = 0, PH_OBS, PH_DRAW, PH_RESOLVE, PH_STORE, PH_DEAL, PH_EPILOGUE, PH_HANDS, PH_APPLY, PH_B1, PH_B2,
    PR_DRAWS, PR_B1, PR_TARGETS, PR_APPLY, PR_HANDS, PR_DRAWS2, PR_B2, PR_STORE, PR_SPARE, PH_N
};
#ifdef SECHS_PHASE_PROF
__device__ unsigned long long g_phase[PH_N + 2];
struct PhaseProf {
    uint64_t t, acc[PH_N];
    __device__ __forceinline__ void start() {
        t = __builtin_readcyclecounter();
#pragma unroll
        for (int k = 0; k < PH_N; k++) acc[k] = 0ull;
    }
    __device__ __forceinline__ void mark(int k) {
        const uint64_t n = __builtin_readcyclecounter();
        acc[k] += n - t;
        t = n;
    }
    __device__ __forceinline__ void flush(int lane, int role = 0) {
        if (lane == 0) {
#pragma unroll
            for (int k = 0; k < PH_N; k++)
                if (acc[k]) atomicAdd(&g_phase[k], (unsigned long long)acc[k]);
            atomicAdd(&g_phase[PH_N + role], 1ull);
        }
    }
};
#else
struct PhaseProf {
    __device__ __forceinline__ void start() {}
    __device__ __forceinline__ void mark(int) {}
    __device__ __forceinline__ void flush(int, int = 0) {}
};
#endif

// MT19937 chunks (8 words) twisted per refill in k_play: 2 doubles the
// lookahead of the refill's loads (one wave per SIMD: nothing else hides them)
constexpr int kPlayPrefetch = 2;

struct PlayArgs {
    int steps, flags, obs_stride, wave_lds;  // wave_lds: bytes of LDS per wave (dynamic)
    int ring_lds;            // bytes of that per lane for the LDS ring copy (RNG_NUMPY_RING/PIPE), at the region's end
    int pipe_cin, pipe_cout, pipe_t;  // RNG_NUMPY_PIPE: pabsc parity read / written, ptend parity read
    int vec_out;             // rewards 16-B and actions 4-B aligned: one store per lane each (N == 4)
    const int32_t* actions;  // [B][N] (steps == 1) or NULL = DrunkHamster
    int32_t* rewards;        // [steps][B][N]
    uint8_t* done;           // [steps][B]
    uint8_t* actions_out;    // [steps][B][N]
    int8_t* obs;             // [steps][B][N][obs_stride]
    int32_t* invalid;        // [B]
    int32_t* league_rec;     // league: [episodes][B][1 + N] per finished game: seats word, results
    int step0;               // league: env-steps of this rollout before this launch (episode index of a record)
    int n0;                  // k_play_split: every game's hand size at the launch's start (aligned handle);
                             // RNG_NUMPY_DEC: the launch's first step within its episode (0..9)
    int drec0, drec1;        // RNG_NUMPY_DEC: record slots of the launch's episode and of the next one
};

// The env-step loop of one lane (game g).  R supplies the random words
// (topup/force, sechs_device.h).  Each wave
// owns a private LDS region: the lanes' deal decks, and -- when the
// observation rows are 48 bytes -- a staging area where the wave's 64 rows
// are assembled so that they leave as 1-KB contiguous stores instead of 64
// scattered 16-B pieces per instruction.  (Both uses never overlap in time
// within a step: observations first, the deal at the very end.)
// Where a step's random decisions come from.  StreamSrc: the game's own
// word stream, in the play loop (DrunkHamster draws, tournament seat draws,
// the deal).  SplitSrc: decisions a producer wave decoded into LDS
// (k_play_split): the indices of every step, the next deal's hands/rows.
template <int N, class R>
struct StreamSrc {
    R& rng;
    ByteBuf& buf;
    uint8_t* deck;  // kDealStride bytes of LDS: deck + swap targets
    __device__ __forceinline__ void draws(const Game<N>& G, int, uint32_t kp, bool lg, uint32_t (&idx)[N]) {
        // DrunkHamster for every seat in seat order (play.py:38-41):
        // legal[random_interval(n-1)], agents/random.py:9
        if (lg && !__all(kp == (uint32_t)N)) {  // a tournament game with fewer players
#pragma unroll
            for (int p = 0; p < N; p++) idx[p] = ((uint32_t)p < kp) ? rng_interval(rng, buf, G.n - 1u) : 0u;
        } else {
            rng_draws<N>(rng, buf, G.n - 1u, idx);
        }
    }
    __device__ __forceinline__ uint32_t league(const DevState& s) { return league_draw(rng, buf, s.lg_K, s.lg_lo, s.lg_hi); }
    __device__ __forceinline__ void deal(const DevState& s, Game<N>& G, PhaseProf& pp) {
        // deck_shuffle2 in its two phases (marked apart for the profiler)
        shuffle_targets(rng, buf, deck + kDeckStride, s.C);
        pp.mark(PH_DEAL);
        for (int i = 0; i < s.C; i += 4) *(uint32_t*)(deck + i) = (uint32_t)i * 0x01010101u + 0x03020100u;
        shuffle_apply(deck, deck + kDeckStride, s.C);
        pp.mark(PH_APPLY);
        deal_from_deck<N>(deck, s.C, G);
#pragma unroll
        for (int p = 0; p < N; p++) SN_DASSERT(hand_strict(G.hand[p]) && hand_len(G.hand[p]) == (uint32_t)kHand);
    }
};

// ---- decode-ahead records (SN_OPT_PIPE_DEC, the default for lockstep
// DrunkHamster rollouts of a numpy-compat handle, N <= 4) -----------------
// Every random decision of such a rollout depends on the word stream only
// (the draw maxima are n - 1 for the known hand size n, the deal's are
// 103..1), so k_decode, on the side stream beside the play launches, walks
// each game's pipelined ring a group of launches ahead and writes one record
// per game and episode; k_play<RNG_NUMPY_DEC> then plays from the records
// and issues no RNG work: no draws, no swap targets, no Fisher-Yates swaps,
// no hand sorting.  Record of an episode, 24 dwords as kDecQuads u32x4
// pieces at drec[(slot * kDecQuads + q) * B + g] (a wave's piece q of 64
// games is one 1-KB run):
//   w0       stream position where the record starts (the first decoded
//            step: step phi0 of the pipeline's first episode, else step 0)
//   w1..w5   off[t], t = 0..9 (u16 pairs): words consumed from w0 through
//            step t's draws (t = 9: through the deal that ends the episode)
//   w6..w10  step t's draws, t = 0..8 (u16 each: seat p's index at bits 4p;
//            step 9 holds one card, numpy draws nothing)
//   w11      the next deal's row cards r0..r3 (bytes, env.py:108-110)
//   w12..w23 the next deal's hands, seat p at w12 + 3p: the sorted legal list
//            as lo32, hi32, hi (bytes 8, 9 | 0xFFFF0000), env.py:104-107
constexpr int kDecWords = 4 * kDecQuads;

__device__ __forceinline__ uint32_t dec_u16(const uint32_t (&w)[kDecWords], int base, int t) {
    // u16 t of the u16 array at dword `base` (t wave-uniform, 0..9)
    uint32_t v = 0u;
#pragma unroll
    for (int k = 0; k < 5; k++) v = (t >> 1 == k) ? w[base + k] : v;
    return (t & 1) ? (v >> 16) : (v & 0xFFFFu);
}

template <int N>
struct DecSrc {
    uint32_t A[kDecWords];  // the launch's episode
    uint32_t B1[11];        // the next episode: w0..w10 (its draws, offsets), when the launch crosses into it
    int phi;                // the launch's first step within its episode

    __device__ __forceinline__ void load(const DevState& s, const PlayArgs& a, int64_t g, bool cross) {
        phi = a.n0;
        const u32x4* ra = s.drec + (int64_t)a.drec0 * kDecQuads * s.B + g;
#pragma unroll
        for (int q = 0; q < kDecQuads; q++) {
            const u32x4 v = ra[(int64_t)q * s.B];
            A[4 * q] = v.x, A[4 * q + 1] = v.y, A[4 * q + 2] = v.z, A[4 * q + 3] = v.w;
        }
#pragma unroll
        for (int k = 0; k < 11; k++) B1[k] = 0u;
        if (cross) {
            const u32x4* rb = s.drec + (int64_t)a.drec1 * kDecQuads * s.B + g;
#pragma unroll
            for (int q = 0; q < 3; q++) {
                const u32x4 v = rb[(int64_t)q * s.B];
                B1[4 * q] = v.x, B1[4 * q + 1] = v.y, B1[4 * q + 2] = v.z;
                if (q < 2) B1[4 * q + 3] = v.w;
            }
        }
    }
    __device__ __forceinline__ void draws(const Game<N>&, int t, uint32_t, bool, uint32_t (&idx)[N]) {
        const int tau = phi + t;  // wave-uniform
        uint32_t v;
        if (tau < kHand) {
            v = (tau < kHand - 1) ? dec_u16(A, 6, tau) : 0u;
        } else {
            uint32_t w[kDecWords];
#pragma unroll
            for (int k = 0; k < kDecWords; k++) w[k] = (k < 11) ? B1[k] : 0u;
            v = (tau - kHand < kHand - 1) ? dec_u16(w, 6, tau - kHand) : 0u;
        }
#pragma unroll
        for (int p = 0; p < N; p++) idx[p] = (v >> (4 * p)) & 15u;
    }
    __device__ __forceinline__ uint32_t league(const DevState&) { return 0u; }
    __device__ __forceinline__ void deal(const DevState&, Game<N>& G, PhaseProf&) {  // the next episode's deal
#pragma unroll
        for (int p = 0; p < N; p++) {
            G.hand[p].lo = (uint64_t)A[12 + 3 * p] | ((uint64_t)A[13 + 3 * p] << 32);
            G.hand[p].hi = A[14 + 3 * p];
            G.score[p] = 0;
        }
        const uint32_t rw = A[11];
        const uint32_t r0 = rw & 0xFFu, r1 = (rw >> 8) & 0xFFu, r2 = (rw >> 16) & 0xFFu, r3 = rw >> 24;
        G.b.lo = u32x4{r0, r1, r2, r3};
        G.b.hi = u32x4{meta_row(r0), meta_row(r1), meta_row(r2), meta_row(r3)};
        G.n = kHand;
    }
    // the stream position after the launch's last step (what sn_pipe_sync exports)
    __device__ __forceinline__ uint32_t position(int steps) const {
        const int last = phi + steps - 1;
        if (last < kHand) return A[0] + dec_u16(A, 1, last);
        uint32_t w[kDecWords];
#pragma unroll
        for (int k = 0; k < kDecWords; k++) w[k] = (k < 11) ? B1[k] : 0u;
        return w[0] + dec_u16(w, 1, last - kHand);
    }
};

// 16-B pieces per lane in the obs staging rows: 3N padded to an odd count, so
// the 64 lanes' ds_write_b128 at a common piece index spread over all banks
// (an even stride -- 12 pieces = 192 B at N = 4 -- serialised them)
__host__ __device__ constexpr int obs_stage_pieces(int N) { return 3 * N + ((N & 1) ? 0 : 1); }

template <int N, class Src, int GPW = 64, bool LG = false>
__device__ __forceinline__ void play_steps(const DevState& s, const PlayArgs& a, int64_t g, int lane, uint8_t* wave_lds,
                                           Game<N>& G, Src& src, int32_t (&sum_res)[N], int32_t& episodes,
                                           PhaseProf& pp, uint32_t& lg, int t_begin, int t_end) {
    const int64_t B = s.B;
    const bool staged = a.obs && a.obs_stride == 48;
    const int64_t g0 = g - lane;                           // first game of this wave
    const int wave_games = (int)min((int64_t)GPW, B - g0);  // = active lanes (lanes past B left)
    const bool auto_reset = (a.flags & SN_AUTO_RESET) != 0;
    const bool summ = !(a.flags & SN_NO_SUMMARIES);
    int32_t* rew = a.rewards ? a.rewards + ((int64_t)t_begin * B + g) * N : nullptr;
    uint8_t* act = a.actions_out ? a.actions_out + ((int64_t)t_begin * B + g) * N : nullptr;
    uint8_t* dn = a.done ? a.done + (int64_t)t_begin * B + g : nullptr;
    int8_t* ob = a.obs ? a.obs + ((int64_t)t_begin * B + g) * N * a.obs_stride : nullptr;
    for (int t = t_begin; t < t_end; t++) {
        const uint32_t kp = LG ? (lg & 15u) : (uint32_t)N;  // players of this game
        if (ob) {
            uint32_t w2hi;
            const int nobs = LG ? (int)kp : N;
            const GameWords gw = summ ? game_words<true>(nobs, G.b, w2hi) : game_words<false>(nobs, G.b, w2hi);
            if (staged) {
                constexpr int P = obs_stage_pieces(N);  // odd: lanes' rows land on distinct bank groups
                u32x4* row = (u32x4*)wave_lds + lane * P;
#pragma unroll
                for (int p = 0; p < N; p++) {
                    const Hand& h = G.hand[p];
                    row[3 * p + 0] = u32x4{(uint32_t)h.lo, (uint32_t)(h.lo >> 32), (h.hi & 0xFFFFu) | w2hi, gw.w0};
                    row[3 * p + 1] = gw.a;
                    row[3 * p + 2] = gw.b;
                }
                __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
                const u32x4* src = (const u32x4*)wave_lds;
                u32x4* dst = (u32x4*)(a.obs + ((int64_t)t * B + g0) * N * 48);
                if (wave_games == GPW) {  // all reads, one wait, all stores
                    u32x4 pc[3 * N];
#pragma unroll
                    for (int j = 0; j < 3 * N; j++) {
                        const int c = lane + GPW * j;  // piece c of the wave's contiguous obs block
                        pc[j] = src[(c / (3 * N)) * P + c % (3 * N)];
                    }
#pragma unroll
                    for (int j = 0; j < 3 * N; j++) {
                        if (SECHS_NT_OBS) __builtin_nontemporal_store(pc[j], &dst[lane + GPW * j]);
                        else dst[lane + GPW * j] = pc[j];
                    }
                } else {
                    const int pieces = wave_games * N * 3;
                    for (int i = lane; i < pieces; i += wave_games) dst[i] = src[(i / (3 * N)) * P + i % (3 * N)];
                }
                __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
            } else {
#pragma unroll
                for (int p = 0; p < N; p++) store_obs_row(ob + p * a.obs_stride, G.hand[p], w2hi, gw, a.obs_stride);
            }
            ob += B * N * a.obs_stride;
        }
        pp.mark(PH_OBS);
        uint32_t card[N], pen[N], idx[N];
        int bad = -1;
        if (G.n == 0u) {
            bad = 0;  // finished game stepped without auto-reset: nothing to play
        } else if (a.actions) {
#pragma unroll
            for (int p = N - 1; p >= 0; p--) {
                const int32_t c = a.actions[g * N + p];
                const int k = (c >= 0 && c < s.C) ? hand_find(G.hand[p], (uint32_t)c) : -1;
                card[p] = (uint32_t)c;
                idx[p] = (uint32_t)k;
                bad = (k >= 0) ? bad : p;
            }
        } else {
            src.draws(G, t, kp, LG, idx);
#pragma unroll
            for (int p = 0; p < N; p++) {
                card[p] = hand_get(G.hand[p], idx[p]);
                SN_DASSERT((LG && (uint32_t)p >= kp) || (idx[p] < G.n && card[p] < (uint32_t)s.C));  // the hand holds it
            }
        }
        pp.mark(PH_DRAW);
        if (a.invalid) a.invalid[g] = bad;
        if (bad >= 0) {
            if (rew) {
#pragma unroll
                for (int p = 0; p < N; p++) rew[p] = 0;
                rew += B * N;
            }
            if (act) act += B * N;
            if (dn) {
                *dn = (G.n == 0u) ? 1 : 0;
                dn += B;
            }
            continue;
        }
#pragma unroll
        for (int p = 0; p < N; p++) hand_del(G.hand[p], idx[p]);
        resolve<N, LG>(G.b, card, pen);  // absent seats' cards are 0xFF (empty hands)
#pragma unroll
        for (int p = 0; p < N; p++) G.score[p] += (int32_t)pen[p];
        G.n -= 1u;
        const bool done = (G.n == 0u);  // env.py:246-249
        pp.mark(PH_RESOLVE);
        if (rew) {
            if (N == 4 && a.vec_out) {  // one 16-B store per lane: 1 KB contiguous per wave
                st_nt((u32x4*)rew, u32x4{-pen[0], -pen[1 % N], -pen[2 % N], -pen[3 % N]}, SECHS_NT_MORE);
            } else {
#pragma unroll
                for (int p = 0; p < N; p++) rew[p] = -(int32_t)pen[p];
            }
            rew += B * N;
        }
        if (act) {
            if (N == 4 && a.vec_out) {
                st_nt((uint32_t*)act, (uint32_t)(card[0] | (card[1 % N] << 8) | (card[2 % N] << 16) | (card[3 % N] << 24)),
                      SECHS_NT_MORE);
            } else {
#pragma unroll
                for (int p = 0; p < N; p++) act[p] = (uint8_t)card[p];
            }
            act += B * N;
        }
        if (dn) {
            st_nt(dn, (uint8_t)(done ? 1 : 0), SECHS_NT_MORE);
            dn += B;
        }
        pp.mark(PH_STORE);
        if (LG && done && a.league_rec) {  // the finished game's record: seats word, results (-penalty)
            int32_t* rec = a.league_rec + ((int64_t)((a.step0 + t) / kHand) * B + g) * (1 + N);
            rec[0] = (int32_t)lg;
#pragma unroll
            for (int p = 0; p < N; p++) rec[1 + p] = -G.score[p];
        }
        if (done && auto_reset) {
            // GameSession.results.append(scores) then the next play_game()
#pragma unroll
            for (int p = 0; p < N; p++) sum_res[p] -= G.score[p];
            episodes += 1;
            if (LG) lg = src.league(s);  // Tournament.play_game: seats first
            src.deal(s, G, pp);
            if (LG) {  // a k-player env deals k hands (env.py:108)
                const uint32_t k2 = lg & 15u;
#pragma unroll
                for (int p = 0; p < N; p++)
                    if ((uint32_t)p >= k2) G.hand[p].lo = ~0ull, G.hand[p].hi = ~0u;
            }
            pp.mark(PH_HANDS);
        }
    }
}

// episode results stay in registers for the launch (one load, one store)
template <int N>
__device__ __forceinline__ void load_results(const DevState& s, int64_t g, int flags, int32_t (&sum_res)[N], int32_t& episodes) {
#pragma unroll
    for (int p = 0; p < N; p++) sum_res[p] = 0;
    episodes = 0;
    if (flags & SN_AUTO_RESET) {
#pragma unroll
        for (int p = 0; p < N; p++) sum_res[p] = s.sum_res[(int64_t)p * s.B + g];
        episodes = s.episodes[g];
    }
}

template <int N>
__device__ __forceinline__ void store_results(const DevState& s, int64_t g, int flags, const int32_t (&sum_res)[N],
                                              int32_t episodes) {
    if (flags & SN_AUTO_RESET) {
#pragma unroll
        for (int p = 0; p < N; p++) s.sum_res[(int64_t)p * s.B + g] = sum_res[p];
        s.episodes[g] = episodes;
    }
}

// GPW = games per wave: 64 (one game per lane), or 32 for the pipelined
// path (lanes 32..63 idle) -- half the LDS per wave, so two blocks fit a CU
// and a SIMD holds two waves to hide each other's latency
template <int N, int MODE, int GPW, bool LG = false>
__device__ __forceinline__ void play_body(const DevState& s, const PlayArgs& a, uint8_t* lds_dyn, int tid) {
    const int lane = tid & 63;
    if (GPW < 64 && lane >= GPW) return;
    // issue priority over the co-resident k_mt_ahead waves: the game loop
    // is one latency-bound wave per SIMD (measured +1.7 %)
    __builtin_amdgcn_s_setprio(1);
    const int64_t g = ((int64_t)blockIdx.x * (kBlock / 64) + (tid >> 6)) * GPW + lane;
    if (g >= s.B) return;
    uint8_t* wave_lds = lds_dyn + (tid >> 6) * a.wave_lds;
    PhaseProf pp;
    pp.start();
    Game<N> G;
    load_game<N>(s, g, G);
    int32_t sum_res[N], episodes;
    load_results<N>(s, g, a.flags, sum_res, episodes);
    uint32_t lg = LG ? s.lgs[g] : 0u;
    ByteBuf buf;
    if constexpr (MODE == RNG_NUMPY_DEC) {
        DecSrc<N> src;
        src.load(s, a, g, a.n0 + a.steps > kHand);
        pp.mark(PH_PROLOGUE);
        play_steps<N, DecSrc<N>, 64, false>(s, a, g, lane, wave_lds, G, src, sum_res, episodes, pp, lg, 0, a.steps);
        s.pabsc[(int64_t)a.pipe_cout * s.B + g] = src.position(a.steps);  // the consumer position (sn_pipe_sync)
    } else if constexpr (MODE == RNG_NUMPY_PIPE) {
        RingPipe rng;
        rng.load(s, g, buf, wave_lds + a.wave_lds - GPW * a.ring_lds + lane * a.ring_lds, a.pipe_cin, a.pipe_t);
        pp.mark(PH_PROLOGUE);
        StreamSrc<N, RingPipe> src{rng, buf, wave_lds + lane * kDealStride};
        play_steps<N, StreamSrc<N, RingPipe>, GPW, LG>(s, a, g, lane, wave_lds, G, src, sum_res, episodes, pp, lg, 0,
                                                       a.steps);
        s.pabsc[(int64_t)a.pipe_cout * s.B + g] = rng.consumed(buf);  // read by k_mt_ahead on the other queue
    } else {
        typename RngOf<MODE, kPlayPrefetch>::T rng;
        if constexpr (MODE == RNG_NUMPY_RING || MODE == RNG_NUMPY_RING_HBM) {
            uint8_t* slot = wave_lds + a.wave_lds - 64 * a.ring_lds + lane * a.ring_lds;
            RngOf<MODE, kPlayPrefetch>::load(s, g, rng, buf, slot);
        } else {
            RngOf<MODE, kPlayPrefetch>::load(s, g, rng, buf);
        }
        pp.mark(PH_PROLOGUE);
        using Gen = typename RngOf<MODE, kPlayPrefetch>::T;
        StreamSrc<N, Gen> src{rng, buf, wave_lds + lane * kDealStride};
        play_steps<N, StreamSrc<N, Gen>, 64, LG>(s, a, g, lane, wave_lds, G, src, sum_res, episodes, pp, lg, 0, a.steps);
        RngOf<MODE, kPlayPrefetch>::store(s, g, rng, buf);
    }
    store_game<N>(s, g, G);
    store_results<N>(s, g, a.flags, sum_res, episodes);
    if (LG) s.lgs[g] = lg;
    pp.mark(PH_EPILOGUE);
    pp.flush(lane);
}

template <int N, int MODE, int GPW = 64, bool LG = false>
__global__ __launch_bounds__(kBlock) void k_play(DevState s, PlayArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds_dyn[];
    play_body<N, MODE, GPW, LG>(s, a, lds_dyn, (int)threadIdx.x);
}

// k_decode: the decode-ahead producer.  One lane per game walks its
// pipelined ring from the decoder position (pabsc[kDecSlot]) and writes the
// records of episodes e0 .. e0 + ne - 1 (slots mod kDecRecords): per step
// the N DrunkHamster draws legal[random_interval(n - 1)] in seat order
// (agents/random.py:9, play.py:38-41; n = 10 - t), after step 9 the next
// deal -- np.random.shuffle(arange(C)) as Fisher-Yates from the end
// (env.py:99-112: j = random_interval(i), i = C-1 .. 1), the swaps in the
// lane's LDS deck, the hands sorted -- and the stream offsets after every
// step.  The same words in the same order as k_play's own draws and deals
// (StreamSrc), so the games are the same.  phi0: the first episode starts at
// that step (a pipeline started mid-episode).  The twist before it on the
// same stream (ptend[tpar]) leads the decoder position by the lead.
struct DecArgs {
    int e0, ne, phi0, tpar;
    int cin, cout;  // pabsc slots of the decoder position read / written
};

// One lane per game.  Per episode the lane copies a RingPipe window of its
// ring (kPipeWin bytes from the decoder position, all loads in flight at
// once) to LDS and reads the words from there -- the draws through the byte
// buffer, the shuffle targets straight from the window by position -- as
// the play kernel's own RingPipe path does.  (Reading the ring from HBM unit
// by unit was twice as slow: the loop's loads waited one by one.)  Per lane
// kPipeSlot bytes (an odd 8-B stride): the window; the swap targets overlay
// its first 104 bytes (target k lands on window byte k while the reads are
// past stream offset 36 + k: every earlier draw took >= 1 word), and the
// deck its bytes 112..219 once the targets are drawn.
constexpr int kDecBlock = 64;  // one wave per workgroup: packs beside the play blocks
constexpr int kDecLane = kPipeSlot;
static_assert(kDecLane % 8 == 0 && (kDecLane / 8) % 2 == 1 && kDecLane >= 112 + 108, "decoder LDS lane");

template <int N>
__global__ __launch_bounds__(kDecBlock) void k_decode(DevState s, DecArgs d) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[kDecBlock * kDecLane];
    const int lane = threadIdx.x & 63;
    const int64_t g = (int64_t)blockIdx.x * kDecBlock + threadIdx.x;
    if (g >= s.B) return;
    const int64_t B = s.B;
    uint8_t* win = lds + threadIdx.x * kDecLane;  // the ring window
    uint8_t* jslot = win;                         // the swap targets, over the window's consumed head
    uint8_t* deck = win + 112;                    // the deck, once the window is dead
    uint32_t pos = s.pabsc[(int64_t)d.cin * B + g];
    const uint32_t tend = s.ptend[(int64_t)d.tpar * B + g];
    PhaseProf pq;
    pq.start();
    for (int i = 0; i < d.ne; i++) {
        const int phi = (i == 0) ? d.phi0 : 0;
        RingPipe rng;
        ByteBuf buf;
        rng.load_at(s, g, buf, win, pos, tend);  // an overrun (pos past tend) counts perr there
        const uint32_t start = pos;
        uint32_t off[5] = {0u, 0u, 0u, 0u, 0u}, dr[5] = {0u, 0u, 0u, 0u, 0u};
        bool big = false;
#pragma unroll
        for (int t = 0; t < kHand - 1; t++) {  // steps 0..8: hand size n = 10 - t, draws random_interval(n - 1)
            if (t >= phi) {
                uint32_t idx[N];
                rng_draws<N>(rng, buf, (uint32_t)(kHand - 1 - t), idx);
                uint32_t v = 0u;
#pragma unroll
                for (int p = 0; p < N; p++) v |= idx[p] << (4 * p);
                dr[t >> 1] |= v << (16 * (t & 1));
                const uint32_t o = rng.consumed(buf) - start;
                big = big || o > 0xFFFFu;
                off[t >> 1] |= (o & 0xFFFFu) << (16 * (t & 1));
            }
        }
        pq.mark(PR_DRAWS);
        // step 9 plays each seat's last card (no draw), then the auto-reset deal
        shuffle_targets(rng, buf, jslot, s.C, kDecLane - 1);  // the window's own form (by position), dummy past it
        pos = rng.consumed(buf);
        pq.mark(PR_TARGETS);
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");  // the window reads before the deck's writes
        for (int k = 0; k < s.C; k += 4) *(uint32_t*)(deck + k) = (uint32_t)k * 0x01010101u + 0x03020100u;
        shuffle_apply(deck, jslot, s.C);
        pq.mark(PR_APPLY);
        Game<N> G;
        deal_from_deck<N>(deck, s.C, G);
        pq.mark(PR_HANDS);
        {
            const uint32_t o = pos - start;
            big = big || o > 0xFFFFu;
            off[4] |= (o & 0xFFFFu) << 16;
        }
        if (big) atomicAdd(s.perr, 1u);  // cannot happen (an episode draws ~200 words); fail loudly
        uint32_t hw[12];
#pragma unroll
        for (int p = 0; p < 4; p++) {
            hw[3 * p] = (p < N) ? (uint32_t)G.hand[p].lo : 0u;
            hw[3 * p + 1] = (p < N) ? (uint32_t)(G.hand[p].lo >> 32) : 0u;
            hw[3 * p + 2] = (p < N) ? G.hand[p].hi : 0u;
        }
        const uint32_t rows = G.b.lo.x | (G.b.lo.y << 8) | (G.b.lo.z << 16) | (G.b.lo.w << 24);
        u32x4* rec = s.drec + (int64_t)((d.e0 + i) % kDecRecords) * kDecQuads * B + g;
        rec[0 * B] = u32x4{start, off[0], off[1], off[2]};
        rec[1 * B] = u32x4{off[3], off[4], dr[0], dr[1]};
        rec[2 * B] = u32x4{dr[2], dr[3], dr[4], rows};
        rec[3 * B] = u32x4{hw[0], hw[1], hw[2], hw[3]};
        rec[4 * B] = u32x4{hw[4], hw[5], hw[6], hw[7]};
        rec[5 * B] = u32x4{hw[8], hw[9], hw[10], hw[11]};
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");  // the deck reads before the next window's writes
        pq.mark(PR_STORE);
    }
    pq.flush(lane, 1);
    s.pabsc[(int64_t)d.cout * B + g] = pos;
}

// ---- one-game fast path (the scalar drop-in SechsNimmtEnv, B == 1) -------
// One launch per env.step / env.reset: the actions arrive as kernel
// arguments, the results (invalid seat, done, rewards, scores, int8 obs rows)
// -- and for a reset the numpy MT19937 state in and out -- go through pinned,
// device-mapped host words, so a call is one launch + one stream sync
// instead of a chain of blocking copies.  Words of hbuf:
constexpr int kH1In = 0;      // [624] key, [624] numpy pos        (sn_reset1 in)
constexpr int kH1Out = 1024;  // [0] invalid, [1] done, [2, 2+N) rewards, [2+N, 2+2N) scores, obs bytes N x 48,
                              // [kH1Trace, +N) per seat: row | undercut << 2 | scored << 3 | penalty << 8 (sn_step1)
constexpr int kH1Trace = 160;  // words into the out block (past 2 + 14 N for N <= 10)
constexpr int kH1Mt = 2048;   // [624] key, [624] code, [625] mt0  (sn_reset1 out)
constexpr int kH1Words = 4096;

struct Acts1 {
    int32_t a[kMaxPlayers];
};

template <int N>
__device__ __forceinline__ void out1_game(const DevState& s, const Game<N>& G, uint32_t* out, int summ) {
#pragma unroll
    for (int p = 0; p < N; p++) out[2 + N + p] = (uint32_t)G.score[p];
    uint32_t w2hi;
    const GameWords gw = summ ? game_words<true>(N, G.b, w2hi) : game_words<false>(N, G.b, w2hi);
    uint32_t* ob = out + 2 + 2 * N;
#pragma unroll
    for (int p = 0; p < N; p++) {
        const Hand& h = G.hand[p];
        const uint32_t row[12] = {(uint32_t)h.lo, (uint32_t)(h.lo >> 32), (h.hi & 0xFFFFu) | w2hi, gw.w0, gw.a.x, gw.a.y,
                                  gw.a.z, gw.a.w, gw.b.x, gw.b.y, gw.b.z, gw.b.w};
#pragma unroll
        for (int i = 0; i < 12; i++) ob[12 * p + i] = row[i];
    }
}

template <int N>
__global__ void k_step1(DevState s, Acts1 acts, uint32_t* hb, int summ) {
    if (threadIdx.x != 0) return;
    uint32_t* out = hb + kH1Out;
    Game<N> G;
    load_game<N>(s, 0, G);
    uint32_t card[N], pen[N], idx[N];
    int bad = -1;
#pragma unroll
    for (int p = N - 1; p >= 0; p--) {  // env.py:114-118 in seat order: the first illegal seat
        const int32_t c = acts.a[p];
        const int k = (G.n > 0u && c >= 0 && c < s.C) ? hand_find(G.hand[p], (uint32_t)c) : -1;
        card[p] = (uint32_t)c;
        idx[p] = (uint32_t)k;
        bad = (k >= 0) ? bad : p;
    }
#pragma unroll
    for (int p = 0; p < N; p++) pen[p] = 0u;
    if (bad < 0) {
#pragma unroll
        for (int p = 0; p < N; p++) hand_del(G.hand[p], idx[p]);
        uint32_t trace[N];
        resolve<N>(G.b, card, pen, trace);
#pragma unroll
        for (int p = 0; p < N; p++) G.score[p] += (int32_t)pen[p];
        G.n -= 1u;
        store_game<N>(s, 0, G);
#pragma unroll
        for (int p = 0; p < N; p++) out[kH1Trace + p] = trace[p];
    } else {  // nothing played: the trace words are 0 (sechs.h), not the previous step's
#pragma unroll
        for (int p = 0; p < N; p++) out[kH1Trace + p] = 0u;
    }
    out[0] = (uint32_t)bad;
    out[1] = (G.n == 0u) ? 1u : 0u;
#pragma unroll
    for (int p = 0; p < N; p++) out[2 + p] = (uint32_t)(-(int32_t)pen[p]);
    out1_game<N>(s, G, out, summ);
}

// sn_reset1, one wave: numpy's (key, pos) arrives in pinned words and is
// imported by all 64 lanes at once into LDS; the 103 Fisher-Yates targets of
// env.py:99-112 (np.random.shuffle: j = random_interval(i), i = C-1 .. 1,
// masked rejection) are decoded 64 stream words per instruction -- a word's
// draw index is its prefix count of accepted words, iterated acceptance ->
// ballot -> v_mbcnt to the fixed point -- with whole 624-word blocks twisted
// in LDS when the stream crosses one (as numpy does); the swaps run on the
// deck held in the wave's registers, one lane deals.  The state goes back in
// numpy's own form (the block holding the consumer + pos): the host
// converts nothing.
template <int N>
__global__ __launch_bounds__(64) void k_reset1(DevState s, uint32_t* hb, int summ) {
    constexpr uint32_t D = kMtN - kMtM;  // 227
    __shared__ uint32_t blk[2 * kMtN];   // the consumer's block, then the next one
    __shared__ __attribute__((aligned(16))) uint8_t slot[kDealStride];
    const uint32_t lane = threadIdx.x;
    const uint32_t C = (uint32_t)s.C, C1 = C - 1u;
    PhaseProf prof;  // libsechs_prof.so only: import / twist / decode / shuffle / deal / out (tools/reset1_prof.py)
    prof.start();
    uint32_t kv[(kMtN + 63) / 64];
#pragma unroll
    for (int q = 0; q < (kMtN + 63) / 64; q++) {  // every lane's host loads in flight at once
        const uint32_t i = 64u * q + lane;
        kv[q] = (i < (uint32_t)kMtN) ? hb[kH1In + i] : 0u;
    }
    const uint32_t pos = __builtin_amdgcn_readfirstlane(hb[kH1In + kMtN]);
#pragma unroll
    for (int q = 0; q < (kMtN + 63) / 64; q++) {
        const uint32_t i = 64u * q + lane;
        if (i < (uint32_t)kMtN) blk[i] = kv[q];
    }
    __syncthreads();
    prof.mark(PR_DRAWS);
    // numpy's twist of blk[0, 624) into blk[624, 1248), in its own order:
    // word j reads old j, j + 1 and j + 397 (j < 227) or new j - 227
    auto twist_next = [&]() {
        for (uint32_t j = lane; j < D; j += 64u) blk[kMtN + j] = mt_mix(blk[j], blk[j + 1u], blk[j + kMtM]);
        __syncthreads();
        for (uint32_t j = D + lane; j < 2u * D; j += 64u) blk[kMtN + j] = mt_mix(blk[j], blk[j + 1u], blk[kMtN + j - D]);
        __syncthreads();
        for (uint32_t j = 2u * D + lane; j < (uint32_t)kMtN - 1u; j += 64u)
            blk[kMtN + j] = mt_mix(blk[j], blk[j + 1u], blk[kMtN + j - D]);
        __syncthreads();
        if (lane == 0u) blk[2 * kMtN - 1] = mt_mix(blk[kMtN - 1], blk[kMtN], blk[kMtN + kMtN - 1 - D]);
        __syncthreads();
    };
    uint32_t dw = pos, o0 = 0u, avail = (uint32_t)kMtN;  // word cursor (from blk[0]), draws done, words in blk
    uint8_t* jslot = slot + kDeckStride;
    while (o0 < C1) {
        while (dw + 64u > avail) {  // the next 64 words: twist (a third block: slide the window first)
            if (avail == 2u * kMtN) {
                uint32_t t[(kMtN + 63) / 64];
#pragma unroll
                for (int q = 0; q < (kMtN + 63) / 64; q++) {
                    const uint32_t i = 64u * q + lane;
                    t[q] = (i < (uint32_t)kMtN) ? blk[kMtN + i] : 0u;
                }
                __syncthreads();
#pragma unroll
                for (int q = 0; q < (kMtN + 63) / 64; q++) {
                    const uint32_t i = 64u * q + lane;
                    if (i < (uint32_t)kMtN) blk[i] = t[q];
                }
                __syncthreads();
                dw -= kMtN;
            }
            prof.mark(PR_TARGETS);
            twist_next();
            prof.mark(PR_SPARE);
            avail = 2u * kMtN;
        }
        const uint32_t x = mt_temper(blk[dw + lane]) & 0xFFu;
        auto eval = [&](uint32_t pre, uint32_t& m) -> bool {
            const uint32_t o = o0 + pre;
            m = (o < C1) ? C1 - o : 1u;  // step o shuffles position i = C-1-o: random_interval(i)
            return o < C1 && (x & (0xFFFFFFFFu >> __builtin_clz(m))) <= m;
        };
        uint32_t m;
        uint64_t Acc = __ballot(eval((lane * 3u) >> 2, m));
        while (true) {
            const uint32_t pre = __builtin_amdgcn_mbcnt_hi((uint32_t)(Acc >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)Acc, 0u));
            const uint64_t A2 = __ballot(eval(pre, m));
            if (A2 == Acc) break;
            Acc = A2;
        }
        const uint32_t pre = __builtin_amdgcn_mbcnt_hi((uint32_t)(Acc >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)Acc, 0u));
        if ((Acc >> lane) & 1ull) {
            (void)eval(pre, m);
            jslot[o0 + pre] = (uint8_t)(x & (0xFFFFFFFFu >> __builtin_clz(m)));
        }
        const uint32_t na = (uint32_t)__popcll(Acc);
        if (o0 + na >= C1) {  // the last draw is in this batch: the consumer stops past its word
            dw += 64u - (uint32_t)__builtin_clzll(Acc);
            break;
        }
        o0 += na;
        dw += 64u;
    }
    __syncthreads();
    prof.mark(PR_TARGETS);
    // the swaps, in numpy's order (step o swaps position i_o = C-1-o with
    // its target j_o), resolved in parallel: v(o), the card step o moves from
    // i_o to j_o, is what an earlier step last moved onto i_o (the latest
    // o' < o with j_o' = i_o), else the card i_o itself -- a chain over
    // earlier steps, resolved by pointer jumping; the final card at i_o is
    // what sat on j_o before step o (the same rule), at position 0 v of the
    // last step targeting 0.  Lane l holds steps l and 64 + l.
    {
        __shared__ int32_t val[128], ptr[128], tail[128];
        __shared__ unsigned long long msk[128];
        const uint32_t oa = lane, ob = 64u + lane;
        const bool va = oa < C1, vb = ob < C1;
        const int32_t ia = (int32_t)(C1 - oa), ib = (int32_t)C1 - (int32_t)ob;
        const int32_t ja = va ? jslot[oa] : -1, jb = vb ? jslot[ob] : -1;
        // the latest earlier step with a given target: per 64-step chunk a
        // mask of the lanes targeting each position (LDS atomic or), the
        // highest lane below mine, else the last one of the chunk before
        tail[lane] = -1, tail[64u + lane] = -1;
        msk[lane] = 0ull, msk[64u + lane] = 0ull;
        __syncthreads();
        const uint64_t below = (1ull << lane) - 1ull;
        if (va) atomicOr(&msk[ja], 1ull << lane);
        __syncthreads();
        uint64_t mj = va ? msk[ja] & below : 0ull, mi = va ? msk[ia] & below : 0ull;
        const int32_t pja = mj ? 63 - (int32_t)__builtin_clzll(mj) : -1;
        const int32_t pia = mi ? 63 - (int32_t)__builtin_clzll(mi) : -1;
        if (va && (msk[ja] >> lane) == 1ull) tail[ja] = (int32_t)lane;  // the chunk's last step onto ja
        __syncthreads();
        if (va) msk[ja] = 0ull;
        __syncthreads();
        if (vb) atomicOr(&msk[jb], 1ull << lane);
        __syncthreads();
        mj = vb ? msk[jb] & below : 0ull, mi = vb ? msk[ib] & below : 0ull;
        const int32_t pjb = mj ? 127 - (int32_t)__builtin_clzll(mj) : (vb ? tail[jb] : -1);
        const int32_t pib = mi ? 127 - (int32_t)__builtin_clzll(mi) : (vb ? tail[ib] : -1);
        const uint64_t z1 = __ballot(vb && jb == 0), z0 = __ballot(va && ja == 0);
        const int32_t last0 = z1 ? 127 - (int32_t)__builtin_clzll(z1) : (z0 ? 63 - (int32_t)__builtin_clzll(z0) : -1);
        // v: resolved values (>= 0) or pointers to earlier steps
        int32_t pa = pia, pb = pib;
        int32_t xa = (pa < 0) ? ia : -1, xb = (pb < 0) ? ib : -1;
        val[oa] = xa, ptr[oa] = pa, val[ob] = xb, ptr[ob] = pb;
        __syncthreads();
        while (__ballot((va && xa < 0) || (vb && xb < 0))) {
            int32_t na = xa, nb = xb, qa = pa, qb = pb;
            if (va && xa < 0) {
                const int32_t w = val[pa];
                if (w >= 0) na = w;
                else qa = ptr[pa];
            }
            if (vb && xb < 0) {
                const int32_t w = val[pb];
                if (w >= 0) nb = w;
                else qb = ptr[pb];
            }
            __syncthreads();
            xa = na, xb = nb, pa = qa, pb = qb;
            val[oa] = xa, ptr[oa] = pa, val[ob] = xb, ptr[ob] = pb;
            __syncthreads();
        }
        const int32_t fa = (pja < 0) ? ja : val[max(pja, 0)], fb = (pjb < 0) ? jb : val[max(pjb, 0)];
        const int32_t f0 = (last0 < 0) ? 0 : val[last0];
        __syncthreads();
        if (va) slot[ia] = (uint8_t)fa;
        if (vb) slot[ib] = (uint8_t)fb;
        if (lane == 0u) slot[0] = (uint8_t)f0;
    }
    __syncthreads();
    prof.mark(PR_APPLY);
    // numpy's state after the deal: the block holding the consumer, pos in 1..624
    const uint32_t b0 = (dw > (uint32_t)kMtN) ? (uint32_t)kMtN : 0u, npos = dw - b0;
    for (uint32_t i = lane; i < (uint32_t)kMtN; i += 64u) {
        const uint32_t v = blk[b0 + i];
        s.mt[i] = v;
        hb[kH1Mt + i] = v;
    }
    if (lane == 0u) {
        prof.mark(PR_STORE);
        Game<N> G;
        deal_from_deck<N>(slot, (int)C, G);
        prof.mark(PR_HANDS);
        store_game<N>(s, 0, G);
        const uint32_t code = mt_code_from_numpy((int)npos);
        s.mt_pos[0] = code;
        uint32_t* out = hb + kH1Out;
        out[0] = 0xFFFFFFFFu;
        out[1] = 0u;
#pragma unroll
        for (int p = 0; p < N; p++) out[2 + p] = 0u;
        out1_game<N>(s, G, out, summ);
        hb[kH1Mt + kMtN] = code;
        hb[kH1Mt + kMtN + 1] = 0u;
        prof.mark(PR_B2);
        prof.flush(0, 1);
    }
}


// ============================================================================
// Role-split k_play (SN_OPT_PLAY_SPLIT, the default for aligned rollouts).
// Every random decision of the DrunkHamster self-play depends on the word
// stream only, never on the cards: the hand size at each step is fixed (the
// games of a handle stay in lockstep after a reset: `phase`), so the
// policy draws' maxima are known, and the deal is a function of the words.
// A block is 4 PLAY waves + 4 PRODUCER waves on the same 256 games (two
// waves per SIMD, where one game per lane leaves one: a single wave issues
// a VALU instruction at most every 4 cycles, two every 2).  Producers decode
// the launch's policy indices into LDS (nibbles), barrier B1, then shuffle
// and deal the next episode and decode the steps after it while the play
// waves play up to the episode's end; barrier B2; play waves install the
// dealt hands and go on.  The play waves issue no RNG work at all.  Philox
// handles only (numpy-compat variants over the pipelined ring were measured
// slower than k_play + k_mt_ahead and removed).
// Same words, same order, same results: every parity test runs this path.
// ============================================================================
template <int N>
struct SplitSrc {
    const uint16_t* idx;  // this lane's column of the producer's [t][64] index words
    __device__ __forceinline__ void draws(const Game<N>&, int t, uint32_t, bool, uint32_t (&out)[N]) {
        const uint32_t v = idx[t * 64];
#pragma unroll
        for (int p = 0; p < N; p++) out[p] = (v >> (4 * p)) & 15u;
    }
    __device__ __forceinline__ uint32_t league(const DevState&) { return 0u; }
    __device__ __forceinline__ void deal(const DevState&, Game<N>&, PhaseProf&) {}  // installed after B2
};

// the policy indices of steps [t_from, t_to): hand size m_first at t_from,
// one less each step (the game's n), N seats in seat order (play.py:38-41)
template <int N, class R>
__device__ __forceinline__ void produce_draws(R& rng, ByteBuf& buf, uint16_t* idx, int t_from, int t_to, int m_first) {
    for (int t = t_from; t < t_to; t++) {
        const int m = m_first - (t - t_from);
        uint32_t v = 0u;
        if (m >= 2) {
            uint32_t d[N];
            rng_draws<N>(rng, buf, (uint32_t)(m - 1), d);
#pragma unroll
            for (int p = 0; p < N; p++) v |= d[p] << (4 * p);
        }
        idx[t * 64] = (uint16_t)v;
    }
}

// LDS of a k_play_split block: play staging | decks | index words | dealt games
__host__ __device__ __forceinline__ int split_deal_words(int N) { return 3 * N + 1; }
__host__ __device__ __forceinline__ size_t split_lds(int N, int steps) {
    return (size_t)4 * 64 * obs_stage_pieces(N) * 16 + (size_t)4 * 64 * kDealStride + (size_t)4 * steps * 64 * 2 +
           (size_t)4 * split_deal_words(N) * 64 * 4;
}

template <int N, int MODE>
__global__ __launch_bounds__(2 * kBlock) void k_play_split(DevState s, PlayArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds_dyn[];
    // the role is wave-uniform: readfirstlane makes it a scalar branch, so each
    // wave runs only its role's code -- and exactly its role's two barriers
    const int tid = (int)threadIdx.x, wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63, w = wave & 3;
    const int64_t g = ((int64_t)blockIdx.x * 4 + w) * 64 + lane;
    const bool live = g < s.B;
    uint8_t* staging = lds_dyn + (size_t)w * 64 * obs_stage_pieces(N) * 16;
    uint8_t* decks = lds_dyn + (size_t)4 * 64 * obs_stage_pieces(N) * 16;
    uint16_t* idx = (uint16_t*)(decks + (size_t)4 * 64 * kDealStride) + (size_t)w * a.steps * 64 + lane;
    uint32_t* dealt = (uint32_t*)((uint8_t*)((uint16_t*)(decks + (size_t)4 * 64 * kDealStride) + (size_t)4 * a.steps * 64)) +
                      (size_t)w * split_deal_words(N) * 64 + lane;
    const int n0 = a.n0;
    const bool deal_in = n0 >= 1 && n0 <= a.steps;  // the episode ends at step n0 - 1 of this launch
    const int tA = deal_in ? n0 : a.steps;
    // B0 hands the play waves the first kSplitEarly steps' indices at once, so
    // they start playing while the producers decode the rest (B1)
    const int tE = min(tA, kSplitEarly);
    if (wave >= 4) {  // ---------------- producer (the critical path: issue priority over the play waves)
        __builtin_amdgcn_s_setprio(1);
        static_assert(MODE == RNG_PHILOX, "k_play_split decodes Philox streams only");
        PhiloxGen rng;
        ByteBuf buf;
        PhaseProf pq;
        pq.start();
        if (live) {
            RngOf<MODE, 2>::load(s, g, rng, buf);
            produce_draws<N>(rng, buf, idx, 0, tE, n0);
        }
        __syncthreads();  // B0: the first steps' indices are in LDS
        if (live) produce_draws<N>(rng, buf, idx, tE, tA, n0 - tE);
        pq.mark(PR_DRAWS);
        __syncthreads();  // B1: every index before the deal is in LDS
        pq.mark(PR_B1);
        if (live && deal_in) {
            uint8_t* deck = decks + (size_t)(w * 64 + lane) * kDealStride;
            Game<N> D;
            shuffle_targets(rng, buf, deck + kDeckStride, s.C);
            pq.mark(PR_TARGETS);
            for (int i = 0; i < s.C; i += 4) *(uint32_t*)(deck + i) = (uint32_t)i * 0x01010101u + 0x03020100u;
            shuffle_apply(deck, deck + kDeckStride, s.C);
            pq.mark(PR_APPLY);
            deal_from_deck<N>(deck, s.C, D);
#pragma unroll
            for (int p = 0; p < N; p++) {
                dealt[(3 * p + 0) * 64] = (uint32_t)D.hand[p].lo;
                dealt[(3 * p + 1) * 64] = (uint32_t)(D.hand[p].lo >> 32);
                dealt[(3 * p + 2) * 64] = D.hand[p].hi;
            }
            dealt[3 * N * 64] = (D.b.lo.x & 0xFFu) | ((D.b.lo.y & 0xFFu) << 8) | ((D.b.lo.z & 0xFFu) << 16) | (D.b.lo.w << 24);
            pq.mark(PR_HANDS);
            produce_draws<N>(rng, buf, idx, tA, a.steps, kHand);
            pq.mark(PR_DRAWS2);
        }
        __syncthreads();  // B2: the deal and the later indices are in LDS
        pq.mark(PR_B2);
        if (live) RngOf<MODE, 2>::store(s, g, rng, buf);
        pq.mark(PR_STORE);
        pq.flush(lane, 1);
        return;
    }
    // -------------------------------------------------------- play
    PhaseProf pp;
    pp.start();
    Game<N> G;
    int32_t sum_res[N], episodes = 0;
    uint32_t lg = 0u;
    if (live) {
        load_game<N>(s, g, G);
        load_results<N>(s, g, a.flags, sum_res, episodes);
    }
    pp.mark(PH_PROLOGUE);
    SplitSrc<N> src{idx};
    __syncthreads();  // B0
    pp.mark(PH_B1);
    if (live) play_steps<N, SplitSrc<N>, 64, false>(s, a, g, lane, staging, G, src, sum_res, episodes, pp, lg, 0, tE);
    __syncthreads();  // B1
    pp.mark(PH_B1);
    if (live) play_steps<N, SplitSrc<N>, 64, false>(s, a, g, lane, staging, G, src, sum_res, episodes, pp, lg, tE, tA);
    pp.mark(PH_EPILOGUE);
    __syncthreads();  // B2
    pp.mark(PH_B2);
    if (live) {
        if (deal_in) {  // the next episode's deal (env.py:99-112), decoded by the producer
#pragma unroll
            for (int p = 0; p < N; p++) {
                G.hand[p].lo = (uint64_t)dealt[(3 * p + 0) * 64] | ((uint64_t)dealt[(3 * p + 1) * 64] << 32);
                G.hand[p].hi = dealt[(3 * p + 2) * 64];
                G.score[p] = 0;
            }
            const uint32_t rw = dealt[3 * N * 64];
            const uint32_t r0 = rw & 0xFFu, r1 = (rw >> 8) & 0xFFu, r2 = (rw >> 16) & 0xFFu, r3 = rw >> 24;
            G.b.lo = u32x4{r0, r1, r2, r3};
            G.b.hi = u32x4{meta_row(r0), meta_row(r1), meta_row(r2), meta_row(r3)};
            G.n = kHand;
        }
        pp.mark(PH_DEAL);
        play_steps<N, SplitSrc<N>, 64, false>(s, a, g, lane, staging, G, src, sum_res, episodes, pp, lg, tA, a.steps);
        store_game<N>(s, g, G);
        store_results<N>(s, g, a.flags, sum_res, episodes);
    }
    pp.mark(PH_EPILOGUE);
    pp.flush(lane);
}

// obs in any dtype, one thread per (game, seat)
template <typename T>
__global__ void k_obs(DevState s, T* out, int stride, int summ) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= s.B * s.N) return;
    const int64_t g = i / s.N;
    const int p = (int)(i - g * s.N);
    const Hand h = load_hand(s, p, g);
    const Board b = load_board(s, g);
    uint32_t w2hi;
    const GameWords gwv = summ ? game_words<true>(s.N, b, w2hi) : game_words<false>(s.N, b, w2hi);
    const uint32_t gw[9] = {gwv.w0, gwv.a.x, gwv.a.y, gwv.a.z, gwv.a.w, gwv.b.x, gwv.b.y, gwv.b.z, gwv.b.w};
    const uint32_t all[12] = {(uint32_t)h.lo, (uint32_t)(h.lo >> 32), (h.hi & 0xFFFFu) | w2hi,
                              gw[0], gw[1], gw[2], gw[3], gw[4], gw[5], gw[6], gw[7], gw[8]};
    T* dst = out + i * stride;
    const int L = summ ? 47 : 35;
#pragma unroll
    for (int wi = 0; wi < 12; wi++)
#pragma unroll
        for (int bi = 0; bi < 4; bi++) {
            const int k = 4 * wi + bi;
            if (k < stride) dst[k] = (k < L) ? (T)(int8_t)((all[wi] >> (8 * bi)) & 0xFFu) : (T)0;
        }
    for (int k = 48; k < stride; k++) dst[k] = (T)0;
}

__global__ void k_hands(DevState s, int8_t* out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= s.B * s.N) return;
    const int64_t g = i / s.N;
    const int p = (int)(i - g * s.N);
    const Hand h = load_hand(s, p, g);
#pragma unroll
    for (int k = 0; k < kHand; k++) out[i * kHand + k] = (int8_t)hand_get(h, (uint32_t)k);
}

__global__ void k_board(DevState s, int8_t* out) {
    const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= s.B) return;
    const Board b = load_board(s, g);
    const uint32_t lo[4] = {b.lo.x, b.lo.y, b.lo.z, b.lo.w};
    const uint32_t hi[4] = {b.hi.x, b.hi.y, b.hi.z, b.hi.w};
#pragma unroll
    for (int r = 0; r < kRows; r++)
#pragma unroll
        for (int i = 0; i < kThreshold; i++)
            out[(g * kRows + r) * kThreshold + i] =
                (i < 5 && (uint32_t)i < len_of(hi[r])) ? (int8_t)card_at(lo[r], hi[r], i < 5 ? i : 0) : (int8_t)-1;
}

__global__ void k_scores(DevState s, int32_t* scores, int32_t* sum_res, int32_t* episodes) {
    const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= s.B) return;
    for (int p = 0; p < s.N; p++) {
        if (scores) scores[g * s.N + p] = s.score[(int64_t)p * s.B + g];
        if (sum_res) sum_res[g * s.N + p] = s.sum_res[(int64_t)p * s.B + g];
    }
    if (episodes) episodes[g] = s.episodes[g];
}

__global__ void k_clear_results(DevState s) {
    const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= s.B) return;
    for (int p = 0; p < s.N; p++) s.sum_res[(int64_t)p * s.B + g] = 0;
    s.episodes[g] = 0;
}

// ============================================================================
// host side / C ABI
// ============================================================================
static thread_local std::string g_err;

namespace sechs {
sn_status set_error(sn_status st, const std::string& msg) {
    g_err = msg;
    return st;
}
}  // namespace sechs

static sn_status fail(sn_status st, const std::string& msg) { return set_error(st, msg); }

extern "C" {

const char* sn_last_error(void) { return g_err.c_str(); }
const char* sn_version(void) { return "sechs-mi355x 0.1 (gfx950)"; }

sn_status sn_create(sn_env** out, int device, int64_t num_games, int num_players, int num_cards, uint64_t seed,
                    uint64_t game_offset, int rng_mode) {
    if (!out) return fail(SN_EINVAL, "out is NULL");
    *out = nullptr;
    if (num_games <= 0) return fail(SN_EINVAL, "num_games must be > 0");
    if (num_players < 1 || num_players > kMaxPlayers) return fail(SN_EINVAL, "num_players must be in 1..10");
    if (num_cards < kHand * num_players + kRows) return fail(SN_EINVAL, "num_cards must be >= 10*num_players + 4");
    if (num_cards > kMaxCards) return fail(SN_EUNSUPPORTED, "num_cards > 104 (the reference's _card_value asserts card < 104)");
    if (rng_mode != SN_RNG_PHILOX && rng_mode != SN_RNG_NUMPY_MT) return fail(SN_EINVAL, "unknown rng_mode");
    HIP_TRY(hipSetDevice(device));
    sn_env* e = new (std::nothrow) sn_env();
    if (!e) return fail(SN_ENOMEM, "host allocation failed");
    e->device = device;
    if (hipDeviceGetAttribute(&e->cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || e->cus < 1) {
        delete e;
        return fail(SN_EHIP, "cannot query the device's CU count");
    }
    DevState& s = e->s;
    s.B = num_games, s.N = num_players, s.C = num_cards, s.rng_mode = rng_mode;
    s.seed = seed, s.game_offset = game_offset;
    const int64_t B = num_games, N = num_players;
    struct {
        void** p;
        size_t bytes;
    } allocs[] = {
        {(void**)&s.hand, sizeof(uint32_t) * N * 3 * B},   {(void**)&s.row_lo, sizeof(uint32_t) * kRows * B},
        {(void**)&s.row_hi, sizeof(uint32_t) * kRows * B}, {(void**)&s.score, sizeof(int32_t) * N * B},
        {(void**)&s.sum_res, sizeof(int32_t) * N * B},     {(void**)&s.episodes, sizeof(int32_t) * B},
        {(void**)&s.mt_pos, sizeof(uint32_t) * B},         {(void**)&s.ctr, sizeof(uint64_t) * B},
        {(void**)&s.mt, rng_mode == SN_RNG_NUMPY_MT ? sizeof(uint32_t) * kMtN * B : 4},
        {(void**)&s.mt0, sizeof(uint32_t) * kMt0Levels * B},  // [0]: newest crossing, then the ones before
    };
    for (auto& a : allocs) {
        if (hipMalloc(a.p, a.bytes) != hipSuccess) {
            sn_destroy(e);
            return fail(SN_ENOMEM, "hipMalloc of device state failed");
        }
        (void)hipMemset(*a.p, 0, a.bytes);
    }
    e->chunk_steps = 10;
    e->pipe = 1;
    e->pipe_gpw = 64;
    e->pipe_lead = kPipeLead;
    e->phase = -1;
    e->play_split = 1;
    // measured: three-phase whole-round twists, the
    // ring in 64-B chunks and one twist per four play launches: 0.0861 ->
    // 0.0775 ms per step same box (K = 1 -> 4; K = 2: 0.0792, 3: 0.0783)
    e->twist_round = 1;
    e->twist_every = 4;
    {
        const char* te = getenv("SECHS_TWIST_EVERY");  // default override (A/B runs of whole legs)
        if (te && atoi(te) >= 1 && atoi(te) <= 5) e->twist_every = atoi(te);
    }
    {
        const char* ps = getenv("SECHS_PIPE_SERIAL");
        e->pipe_serial = (ps && ps[0] == '1') ? 1 : 0;
    }
    e->pipe_dec = 1;  // decode-ahead where it applies: 0.0776 -> 0.069 ms per step same box
    {
        const char* pd = getenv("SECHS_PIPE_DEC");  // default override (A/B runs of whole legs)
        if (pd && (pd[0] == '0' || pd[0] == '1')) e->pipe_dec = pd[0] - '0';
    }
    e->pvalid = 0;
    e->pcount = 0;
    if (rng_mode == SN_RNG_NUMPY_MT) {
        struct {
            void** p;
            size_t bytes;
        } pal[] = {{(void**)&s.pring, (size_t)kPipeRing * B},
                   {(void**)&s.pabsc, sizeof(uint32_t) * (kPipeSlots + 2) * B},  // + the decoder's two slots
                   {(void**)&s.ptend, sizeof(uint32_t) * kPipeSlots * B}, {(void**)&s.ptp, sizeof(uint32_t) * B},
                   {(void**)&s.perr, sizeof(uint32_t)},
                   {(void**)&s.drec, N <= kSplitMaxPlayers ? sizeof(u32x4) * kDecRecords * kDecQuads * B : 16}};
        for (auto& a : pal) {
            if (hipMalloc(a.p, a.bytes) != hipSuccess) {
                sn_destroy(e);
                return fail(SN_ENOMEM, "hipMalloc of the MT pipeline failed");
            }
            (void)hipMemset(*a.p, 0, a.bytes);
        }
        // the pipeline's events order kernels on one device only: a device-scope
        // release is enough (the default system-scope one writes L2 back at
        // every record; SECHS_EV_SYSFENCE=1 restores it for A/B runs)
        const char* sf = getenv("SECHS_EV_SYSFENCE");
        const unsigned evf = hipEventDisableTiming | ((sf && sf[0] == '1') ? 0u : (unsigned)hipEventDisableSystemFence);
        if (hipStreamCreateWithFlags(&e->side, hipStreamNonBlocking) != hipSuccess ||
            hipStreamCreateWithFlags(&e->side2, hipStreamNonBlocking) != hipSuccess ||
            hipEventCreateWithFlags(&e->ev_prep2, evf) != hipSuccess ||
            hipEventCreateWithFlags(&e->ev_prep, evf) != hipSuccess ||
            hipEventCreateWithFlags(&e->ev_main, evf) != hipSuccess ||
            hipEventCreateWithFlags(&e->ev_play, evf) != hipSuccess) {
            sn_destroy(e);
            return fail(SN_EHIP, "stream/event creation failed");
        }
        for (int k = 0; k < 2; k++)
            if (hipEventCreateWithFlags(&e->evt[k], evf) != hipSuccess ||
                hipEventCreateWithFlags(&e->evd[k], evf) != hipSuccess) {
                sn_destroy(e);
                return fail(SN_EHIP, "stream/event creation failed");
            }
        if (hipHostMalloc((void**)&e->perr_host, sizeof(uint32_t), hipHostMallocMapped) != hipSuccess ||
            hipHostGetDevicePointer((void**)&e->perr_host_dev, e->perr_host, 0) != hipSuccess) {
            sn_destroy(e);
            return fail(SN_ENOMEM, "pinned overrun mirror allocation failed");
        }
        *e->perr_host = 0u;
    }
    if (rng_mode == SN_RNG_NUMPY_MT) {
        const sn_status r = sn_set_option(e, SN_OPT_RING_WORDS, N <= 4 ? 256 : 512);
        if (r != SN_OK) {
            sn_destroy(e);
            return r;
        }
    }
    hipLaunchKernelGGL(k_seed, dim3(grid_for(B)), dim3(kBlock), 0, 0, s);
    hipError_t err = hipDeviceSynchronize();
    if (err == hipSuccess) err = hipGetLastError();
    if (err != hipSuccess) {
        sn_destroy(e);
        return fail(SN_EHIP, std::string("seeding failed: ") + hipGetErrorString(err));
    }
    *out = e;
    return SN_OK;
}

static void free_timing(sn_env* e);

sn_status sn_destroy(sn_env* e) {
    if (!e) return SN_OK;
    (void)hipSetDevice(e->device);
    DevState& s = e->s;
    (void)hipDeviceSynchronize();  // no k_mt_ahead may still be in flight
    if (e->ev_prep) (void)hipEventDestroy(e->ev_prep);
    if (e->ev_main) (void)hipEventDestroy(e->ev_main);
    if (e->ev_play) (void)hipEventDestroy(e->ev_play);
    for (int k = 0; k < 2; k++) {
        if (e->evt[k]) (void)hipEventDestroy(e->evt[k]);
        if (e->evd[k]) (void)hipEventDestroy(e->evd[k]);
    }
    if (e->ev_prep2) (void)hipEventDestroy(e->ev_prep2);
    if (e->side2) (void)hipStreamDestroy(e->side2);
    if (e->perr_host) (void)hipHostFree(e->perr_host);
    if (e->hbuf) (void)hipHostFree(e->hbuf);
    if (e->side) (void)hipStreamDestroy(e->side);
    free_timing(e);
    void* ps[] = {s.hand, s.row_lo, s.row_hi, s.score, s.sum_res, s.episodes, s.mt_pos, s.ctr, s.mt, s.mt0, s.ring,
                  s.pring, s.pabsc, s.ptend, s.ptp, s.perr, s.lgs, s.lmem, s.drec};
    for (void* p : ps)
        if (p) (void)hipFree(p);
    delete e;
    return SN_OK;
}

static void free_timing(sn_env* e) {
    for (int i = 0; i < kTimingEvents * e->tcap; i++)
        if (e->tev[i]) (void)hipEventDestroy(e->tev[i]);
    delete[] e->tev;
    delete[] e->tev_tw;
    e->tev = nullptr;
    e->tev_tw = nullptr;
    e->tcap = e->tn = 0;
}

sn_status sn_set_option(sn_env* e, int option, int value) {
    if (!e) return fail(SN_EINVAL, "env is NULL");
    DevState& s = e->s;
    if (sn_pipe_sync(e, 0) != SN_OK) return SN_EHIP;
    switch (option) {
        case SN_OPT_RING_WORDS: {
            if (value < 0 || value > 512 || (value % 64)) return fail(SN_EINVAL, "ring words must be a multiple of 64 in 0..512");
            if (value && s.rng_mode != SN_RNG_NUMPY_MT) return fail(SN_EINVAL, "the ring feeds numpy-compat mode only");
            HIP_TRY(hipSetDevice(e->device));
            HIP_TRY(hipDeviceSynchronize());
            if (s.ring) (void)hipFree(s.ring);
            s.ring = nullptr;
            s.ring_w = 0;
            if (value) {
                if (hipMalloc((void**)&s.ring, (size_t)value * (size_t)s.B) != hipSuccess) return fail(SN_ENOMEM, "ring allocation failed");
                s.ring_w = value;
            }
            return SN_OK;
        }
        case SN_OPT_CHUNK_STEPS:
            if (value < 1) return fail(SN_EINVAL, "chunk steps must be >= 1");
            e->chunk_steps = value;
            return SN_OK;
        case SN_OPT_PIPELINE:
            if (value != 0 && value != 1) return fail(SN_EINVAL, "pipeline must be 0 or 1");
            e->pipe = value;
            return SN_OK;
        case SN_OPT_PIPE_GPW:
            if (value != 32 && value != 64) return fail(SN_EINVAL, "games per wave must be 32 or 64");
            e->pipe_gpw = value;
            return SN_OK;
        case SN_OPT_PLAY_SPLIT:
            if (value < 0 || value > 1) return fail(SN_EINVAL, "play split must be 0 or 1");
            e->play_split = value;
            return SN_OK;
        case SN_OPT_TWIST_EVERY:
            if (value < 1 || value > 5) return fail(SN_EINVAL, "twist every must be 1 .. 5");
            e->twist_every = value;
            return SN_OK;
        case SN_OPT_TWIST_ROUND:
            if (value < 0 || value > 1) return fail(SN_EINVAL, "twist round must be 0 or 1");
            e->twist_round = value;
            return SN_OK;
        case SN_OPT_PLAY_QUAD:
        case SN_OPT_PIPE_FUSED:  // round-5 experiments, measured slower and removed
            return fail(SN_EUNSUPPORTED, "option removed (k_play_quad / the fused twist measured slower)");
        case SN_OPT_PIPE_DEC:
            if (value < 0 || value > 1) return fail(SN_EINVAL, "pipe dec must be 0 or 1");
            e->pipe_dec = value;
            return SN_OK;
        case SN_OPT_TWIST_SKIP:
            if (value < 0 || value > 1) return fail(SN_EINVAL, "twist skip must be 0 or 1");
            e->twist_skip = value;
            return SN_OK;
        case SN_OPT_PIPE_LEAD:
            if (value < 64 || value > kPipeLead) return fail(SN_EINVAL, "pipe lead must be in 64..600");
            e->pipe_lead = value;
            return SN_OK;
        case SN_OPT_TIMING:
            if (value < 0 || value > 4096) return fail(SN_EINVAL, "timing launches must be in 0..4096");
            HIP_TRY(hipSetDevice(e->device));
            HIP_TRY(hipDeviceSynchronize());
            free_timing(e);
            if (value) {
                e->tev = new hipEvent_t[kTimingEvents * value]();
                e->tev_tw = new int[value]();
                e->tcap = value;
                for (int i = 0; i < kTimingEvents * value; i++) HIP_TRY(hipEventCreate(&e->tev[i]));
            }
            return SN_OK;
        default: return fail(SN_EINVAL, "unknown option");
    }
}

sn_status sn_info(const sn_env* e, int64_t* B, int* N, int* C, int* mode) {
    if (!e) return fail(SN_EINVAL, "env is NULL");
    if (B) *B = e->s.B;
    if (N) *N = e->s.N;
    if (C) *C = e->s.C;
    if (mode) *mode = e->s.rng_mode;
    return SN_OK;
}

sn_status sn_reset(sn_env* e, const uint8_t* decks, void* stream) {
    if (!e) return fail(SN_EINVAL, "env is NULL");
    hipStream_t st = (hipStream_t)stream;
    if (sn_pipe_sync(e, st) != SN_OK) return SN_EHIP;
    const DevState& s = e->s;
    if (s.lg_K) {  // a batched tournament: every game draws its seats, then deals (tournament.py:132-138)
        if (decks) return fail(SN_EINVAL, "a tournament handle deals from its own streams (decks must be NULL)");
        if (s.rng_mode == SN_RNG_NUMPY_MT) {
            SN_DISPATCH_N(s.N, {
                if constexpr (NN >= 2 && NN <= kLeagueMaxPlayers)
                    hipLaunchKernelGGL((k_reset<NN, RNG_NUMPY_MT, true>), dim3(grid_for(s.B)), dim3(kBlock), 0, st, s, decks);
            });
        } else {
            SN_DISPATCH_N(s.N, {
                if constexpr (NN >= 2 && NN <= kLeagueMaxPlayers)
                    hipLaunchKernelGGL((k_reset<NN, RNG_PHILOX, true>), dim3(grid_for(s.B)), dim3(kBlock), 0, st, s, decks);
            });
        }
        e->lg_phase = 0;
        e->phase = -1;
    } else if (s.rng_mode == SN_RNG_NUMPY_MT) {
        SN_DISPATCH_N(s.N, hipLaunchKernelGGL((k_reset<NN, RNG_NUMPY_MT>), dim3(grid_for(s.B)), dim3(kBlock), 0, st, s, decks));
    } else {
        SN_DISPATCH_N(s.N, hipLaunchKernelGGL((k_reset<NN, RNG_PHILOX>), dim3(grid_for(s.B)), dim3(kBlock), 0, st, s, decks));
    }
    if (!s.lg_K) e->phase = 0;  // every game dealt: in lockstep
    HIP_TRY(hipGetLastError());
    return SN_OK;
}

sn_status sn_reset_to(sn_env* e, const int8_t* board, const int8_t* hands, void* stream) {
    if (!e || !board || !hands) return fail(SN_EINVAL, "NULL argument");
    e->phase = -1;
    hipStream_t st = (hipStream_t)stream;
    const DevState& s = e->s;
    SN_DISPATCH_N(s.N, hipLaunchKernelGGL((k_reset_to<NN>), dim3(grid_for(s.B)), dim3(kBlock), 0, st, s, board, hands));
    HIP_TRY(hipGetLastError());
    return SN_OK;
}

// LDS per CU (gfx950); a k_play block (4 waves) must fit in it
constexpr int kLdsBytes = 160 * 1024;

// k_play_split applies to in-kernel DrunkHamster rollouts of a handle whose
// games are in lockstep (e->phase), with auto-reset, N <= kSplitMaxPlayers
static bool split_ok(const sn_env* e, const PlayArgs& a) {
    return e->play_split && e->phase >= 0 && (a.flags & SN_AUTO_RESET) && !a.actions && !a.invalid && !e->s.lg_K &&
           e->s.N <= kSplitMaxPlayers && !(a.obs && a.obs_stride == 48 && (((uintptr_t)a.obs) & 15));
}

static sn_status launch_play_one(sn_env* e, PlayArgs a, hipStream_t st) {
    const DevState& s = e->s;
    const bool ring = (s.rng_mode == SN_RNG_NUMPY_MT) && !a.actions && s.ring_w > 0;
    int wave = 64 * kDealStride;
    if (a.obs && a.obs_stride == 48 && (((uintptr_t)a.obs) & 15) == 0) wave = max(wave, 64 * obs_stage_pieces(s.N) * 16);
    a.ring_lds = 0;
    const int ring_stride = ring_lds_stride(s.ring_w);
    const bool ring_in_lds = ring && (wave + 64 * ring_stride) * (kBlock / 64) <= kLdsBytes;
    if (ring_in_lds) {
        a.ring_lds = ring_stride;
        wave += 64 * ring_stride;
    }
    a.wave_lds = wave;
    a.vec_out = ((((uintptr_t)a.rewards) & 15) == 0) && ((((uintptr_t)a.actions_out) & 3) == 0);
    const size_t shmem = (size_t)wave * (kBlock / 64);
    if (a.obs && a.obs_stride == 48 && (((uintptr_t)a.obs) & 15)) return fail(SN_EINVAL, "obs with stride 48 must be 16-byte aligned");
    if (ring) {
        constexpr int GPW = kPrepGamesPerWave;
        const dim3 pg((unsigned)((s.B + GPW * (kBlock / 64) - 1) / (GPW * (kBlock / 64))));
        switch (s.ring_w / 64) {
            case 1: hipLaunchKernelGGL((k_mt_prep<1, GPW>), pg, dim3(kBlock), 0, st, s); break;
            case 2: hipLaunchKernelGGL((k_mt_prep<2, GPW>), pg, dim3(kBlock), 0, st, s); break;
            case 3: hipLaunchKernelGGL((k_mt_prep<3, GPW>), pg, dim3(kBlock), 0, st, s); break;
            case 4: hipLaunchKernelGGL((k_mt_prep<4, GPW>), pg, dim3(kBlock), 0, st, s); break;
            case 5: hipLaunchKernelGGL((k_mt_prep<5, GPW>), pg, dim3(kBlock), 0, st, s); break;
            case 6: hipLaunchKernelGGL((k_mt_prep<6, GPW>), pg, dim3(kBlock), 0, st, s); break;
            case 7: hipLaunchKernelGGL((k_mt_prep<7, GPW>), pg, dim3(kBlock), 0, st, s); break;
            case 8: hipLaunchKernelGGL((k_mt_prep<8, GPW>), pg, dim3(kBlock), 0, st, s); break;
            default: return fail(SN_EINVAL, "bad ring size");
        }
        if (ring_in_lds) {
            SN_DISPATCH_N(s.N, {
                HIP_TRY(hipFuncSetAttribute((const void*)k_play<NN, RNG_NUMPY_RING>,
                                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)shmem));
                hipLaunchKernelGGL((k_play<NN, RNG_NUMPY_RING>), dim3(grid_for(s.B)), dim3(kBlock), shmem, st, s, a);
            });
        } else {
            SN_DISPATCH_N(s.N, {
                HIP_TRY(hipFuncSetAttribute((const void*)k_play<NN, RNG_NUMPY_RING_HBM>,
                                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)shmem));
                hipLaunchKernelGGL((k_play<NN, RNG_NUMPY_RING_HBM>), dim3(grid_for(s.B)), dim3(kBlock), shmem, st, s, a);
            });
        }
    } else if (s.rng_mode == SN_RNG_NUMPY_MT) {
        SN_DISPATCH_N(s.N, {
            HIP_TRY(hipFuncSetAttribute((const void*)k_play<NN, RNG_NUMPY_MT>,
                                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)shmem));
            hipLaunchKernelGGL((k_play<NN, RNG_NUMPY_MT>), dim3(grid_for(s.B)), dim3(kBlock), shmem, st, s, a);
        });
    } else if (split_ok(e, a) && a.steps <= kHand) {  // at most one deal per launch
        a.n0 = kHand - e->phase;
        SN_DISPATCH_N(s.N, {
            if constexpr (NN <= kSplitMaxPlayers) {
                const size_t sl = split_lds(NN, a.steps);
                HIP_TRY(hipFuncSetAttribute((const void*)k_play_split<NN, RNG_PHILOX>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                            (int)sl));
                hipLaunchKernelGGL((k_play_split<NN, RNG_PHILOX>), dim3(grid_for(s.B)), dim3(2 * kBlock), sl, st, s, a);
            }
        });
    } else {
        SN_DISPATCH_N(s.N, {
            if (s.lg_K) {
                if constexpr (NN >= 2 && NN <= kLeagueMaxPlayers) {
                    HIP_TRY(hipFuncSetAttribute((const void*)k_play<NN, RNG_PHILOX, 64, true>,
                                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)shmem));
                    hipLaunchKernelGGL((k_play<NN, RNG_PHILOX, 64, true>), dim3(grid_for(s.B)), dim3(kBlock), shmem, st, s, a);
                }
            } else {
                HIP_TRY(hipFuncSetAttribute((const void*)k_play<NN, RNG_PHILOX>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                            (int)shmem));
                hipLaunchKernelGGL((k_play<NN, RNG_PHILOX>), dim3(grid_for(s.B)), dim3(kBlock), shmem, st, s, a);
            }
        });
    }
    HIP_TRY(hipGetLastError());
    return SN_OK;
}

// A ring-fed (numpy-MT, in-kernel DrunkHamster) rollout runs in launches of
// at most chunk_steps env-steps, each behind its own k_mt_prep, so that one
// ring covers a launch's draws (a 4-player episode: 193.5 +- 9.3 words).
sn_status sn_pipe_sync(sn_env* e, hipStream_t st) {
    if (!e || !e->pvalid) return SN_OK;
    // k_pipe_code reads the last k_play's consumer position (pabsc) and the
    // last k_mt_ahead's twisted end: wait for both, whatever stream `st` is
    // (the null stream does not order behind a non-blocking caller stream).
    // ev_play was recorded behind the last pipelined k_play when its rollout
    // was enqueued (launch_pipe), on the caller's stream of that call -- so no
    // stream of an earlier call is touched here; ev_prep is recorded now,
    // behind everything enqueued so far on the side stream.
    HIP_TRY(hipStreamWaitEvent(st, e->ev_play, 0));
    HIP_TRY(hipEventRecord(e->ev_prep, e->side));
    HIP_TRY(hipStreamWaitEvent(st, e->ev_prep, 0));
    HIP_TRY(hipEventRecord(e->ev_prep2, e->side2));  // the decodes (their ring reads) are done too
    HIP_TRY(hipStreamWaitEvent(st, e->ev_prep2, 0));
    // the last play launch wrote pabsc[pl_cout]; the last twist ptend[tw_out]
    hipLaunchKernelGGL(k_pipe_code, dim3((unsigned)((e->s.B + kBlock / 64 - 1) / (kBlock / 64))), dim3(kBlock), 0, st,
                       e->s, e->pl_cout, e->tw_out);
    HIP_TRY(hipGetLastError());
    e->pvalid = 0;
    return SN_OK;
}

// Longest pipelined launch for N players.  k_mt_ahead leaves 593..600 words
// twisted past the consumer position of the launch BEFORE the running one,
// so two consecutive launches must draw <= 592 words.  With auto-reset, 2c
// consecutive env-steps hold at most ceil(2c/10) deals (103 draws each,
// ~146 words) and each hand size at most that often; the exact tail of the
// summed geometric word counts (tools/pipe_tail.py) gives, per game and
// launch pair, P(> 592 words) = 2e-31 at N = 4 with 10-step launches
// (two episodes) but 1.4e-25 at N = 5 and 4.5e-5 at N = 10; with 5-step
// launches (one episode per pair) it is <= 6.1e-73 for every N <= 10.
static int pipe_max_chunk(int N) { return N <= 4 ? 10 : 5; }

// LDS a pipelined k_play block needs (obs staging / deck + the RingPipe windows)
static size_t pipe_lds(const DevState& s, const PlayArgs& a, int gpw, int* wave_out) {
    int wave = gpw * kDealStride;
    if (a.obs && a.obs_stride == 48 && (((uintptr_t)a.obs) & 15) == 0) wave = max(wave, gpw * obs_stage_pieces(s.N) * 16);
    wave += gpw * kPipeSlot;
    *wave_out = wave;
    return (size_t)wave * (kBlock / 64);
}

// one pipelined play launch
static sn_status pipe_play(const DevState& s, const PlayArgs& c, int gpw, unsigned nblk, size_t shmem, hipStream_t st) {
    SN_DISPATCH_N(s.N, {
        if (gpw == 32) {
            HIP_TRY(hipFuncSetAttribute((const void*)k_play<NN, RNG_NUMPY_PIPE, 32>,
                                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)shmem));
            hipLaunchKernelGGL((k_play<NN, RNG_NUMPY_PIPE, 32>), dim3(nblk), dim3(kBlock), shmem, st, s, c);
        } else if (s.lg_K) {
            if constexpr (NN >= 2 && NN <= kLeagueMaxPlayers) {
                HIP_TRY(hipFuncSetAttribute((const void*)k_play<NN, RNG_NUMPY_PIPE, 64, true>,
                                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)shmem));
                hipLaunchKernelGGL((k_play<NN, RNG_NUMPY_PIPE, 64, true>), dim3(nblk), dim3(kBlock), shmem, st, s, c);
            }
        } else {
            HIP_TRY(hipFuncSetAttribute((const void*)k_play<NN, RNG_NUMPY_PIPE>,
                                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)shmem));
            hipLaunchKernelGGL((k_play<NN, RNG_NUMPY_PIPE>), dim3(nblk), dim3(kBlock), shmem, st, s, c);
        }
    });
    HIP_TRY(hipGetLastError());
    return SN_OK;
}

// The pipelined numpy-MT rollout: per launch of <= 10 env-steps, k_play (on
// the caller's stream) draws from words k_mt_ahead twisted during the
// previous launch, while the next k_mt_ahead runs on the side stream.
// Hand-off: HIP events both ways -- a wait and a record on the caller's
// stream between play launches.  (Device-flag and in-launch hand-offs were
// built and measured slower on gfx950)
// one decode-ahead play launch (RNG_NUMPY_DEC: N <= 4, 64 games per wave)
static sn_status dec_play(const DevState& s, const PlayArgs& c, size_t shmem, hipStream_t st) {
    SN_DISPATCH_N(s.N, {
        if constexpr (NN <= kSplitMaxPlayers) {
            HIP_TRY(hipFuncSetAttribute((const void*)k_play<NN, RNG_NUMPY_DEC>,
                                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)shmem));
            hipLaunchKernelGGL((k_play<NN, RNG_NUMPY_DEC>), dim3(grid_for(s.B)), dim3(kBlock), shmem, st, s, c);
        }
    });
    HIP_TRY(hipGetLastError());
    return SN_OK;
}

// records of episodes [e0, e0 + ne) (global counter since the pipeline start) on stream st
static sn_status dec_launch(sn_env* e, int64_t e0, int ne, int phi0, int tpar, int cin, int cout, hipStream_t st) {
    const DevState& s = e->s;
    const DecArgs d{(int)(e0 % kDecRecords), ne, phi0, tpar, cin, cout};
    const dim3 grid((unsigned)((s.B + kDecBlock - 1) / kDecBlock));
    SN_DISPATCH_N(s.N, {
        if constexpr (NN <= kSplitMaxPlayers) hipLaunchKernelGGL((k_decode<NN>), grid, dim3(kDecBlock), 0, st, s, d);
    });
    HIP_TRY(hipGetLastError());
    return SN_OK;
}

// Decode-ahead applies to in-kernel DrunkHamster rollouts with auto-reset of
// a plain (non-tournament) handle of N <= 4 whose games are in lockstep
// (e->phase known): every launch's random decisions are then the same
// function of the stream for every game.
static bool dec_ok(const sn_env* e, const PlayArgs& a) {
    return e->pipe_dec && e->phase >= 0 && (a.flags & SN_AUTO_RESET) && !a.actions && !a.invalid && !e->s.lg_K &&
           e->s.N <= kSplitMaxPlayers && e->pipe_gpw == 64 && e->s.drec;
}

static sn_status launch_pipe(sn_env* e, PlayArgs a, hipStream_t st) {
    DevState& s = e->s;
    int wave;
    const int gpw = e->pipe_gpw;
    const bool dec = dec_ok(e, a);
    size_t shmem = pipe_lds(s, a, gpw, &wave);
    a.ring_lds = kPipeSlot;
    if (dec) {  // the obs staging only (no deck, no ring window)
        wave = (a.obs && a.obs_stride == 48 && (((uintptr_t)a.obs) & 15) == 0) ? 64 * obs_stage_pieces(s.N) * 16 : 16;
        shmem = (size_t)wave * (kBlock / 64);
        a.ring_lds = 0;
    }
    a.wave_lds = wave;
    a.vec_out = ((((uintptr_t)a.rewards) & 15) == 0) && ((((uintptr_t)a.actions_out) & 3) == 0);
    const dim3 pg((unsigned)((s.B + kBlock / 64 - 1) / (kBlock / 64)));
    const int64_t B = s.B, N = s.N;
    // SN_OPT_TWIST_EVERY = K: play launches in groups of K; beside the first
    // launch p of group G runs twist G, leading the consumer position of
    // launch p-1 by 600 K words -- the 2K launches p .. p+2K-1, i.e. K
    // launch pairs of the §4 tail bound -- and launch p waits for twist G-1
    // only, which had a whole group of launches to finish.  Per group, one
    // record and one wait on the caller's stream (K = 1: the launch before).
    // Slots: pabsc by launch index mod kPipeSlots (8 >= K + 3: the next writer
    // of launch p-1's slot is launch p+7, in group G+1 or later, which is
    // ordered behind twist G -- the reader of that slot), ptend by group
    // parity (INIT = launch -1 / twist -1).  The ring holds the lead + a round
    // for K <= 5 (3 623 words), and mt0 the five word-0 crossings that span.
    const int K = e->twist_every;
    const bool round_tw = e->twist_round;
    if (e->pvalid && (e->pK != K || (e->pdec != 0) != dec)) {  // restart with the other group size / form
        const sn_status r = sn_pipe_sync(e, st);
        if (r != SN_OK) return r;
    }
    // Decode-ahead: twist G runs on `side` CONCURRENTLY with decode G on `side2`, so it leads
    // the decoder position after decode G-1 (slot kDecSlot + ((G - 1) & 1)) by the words of
    // the 2K + 1 episodes decode G+1 may need: 600 (K + 1) words (~200 per episode at N <= 4;
    // the ring holds the lead + a round up to 3 472), and the play launches read no ring at
    // all.  Otherwise the twists lead the play consumer by 600 K words.
    const int lead = dec ? min(e->pipe_lead * (K + 1), kPipeRing - kMtN) : e->pipe_lead * K;
    constexpr uint32_t kSlotMask = (uint32_t)kPipeSlots - 1u;
    if (!e->pvalid) {  // start the pipeline from mt_pos: twist the lead ahead, synchronously
        // decode-ahead: the start position to the decoder's input slot of the first decode and
        // the play slot (a sync before any play launch exports it)
        const AheadArgs aa{dec ? kDecSlot : (int)kSlotMask, 0, 1, lead, e->perr_host_dev, dec ? (int)kSlotMask : -1};
        e->tw_out = 1, e->pl_cout = (int)kSlotMask, e->pphase = 0;
        if (round_tw) hipLaunchKernelGGL((k_mt_ahead<true, true>), pg, dim3(kBlock), 0, st, s, aa);
        else hipLaunchKernelGGL((k_mt_ahead<true, false>), pg, dim3(kBlock), 0, st, s, aa);
        HIP_TRY(hipGetLastError());
        if (dec) {  // the records of the first group's launches (episodes 0 .. K), from the current step on
            e->dec_e = 0;
            const sn_status r = dec_launch(e, 0, K + 1, e->phase, 1, kDecSlot, kDecSlot + 1, st);  // "decode -1"
            if (r != SN_OK) return r;
            e->dec_next = K + 1;
        }
        HIP_TRY(hipEventRecord(e->ev_prep, st));
        e->pvalid = 1;
        e->pK = K;
        e->pdec = dec ? 1 : 0;
    } else {
        // order behind the last pipelined k_play (recorded on the stream of
        // that call): always, also on the same stream -- a stream handle's
        // value may be reused by a new stream once the caller destroyed the
        // old one, and a wait on an event already behind costs ~nothing
        HIP_TRY(hipStreamWaitEvent(st, e->ev_play, 0));
    }
    // a tournament game adds its seat draw (<= K - 1 + 1 draws): 10-step
    // launches keep the pair tail < 1e-26 up to K = 8 agents at N <= 4
    // (tools/pipe_tail.py), beyond that 5-step launches
    const int chunk = min(e->chunk_steps, (s.lg_K > 8) ? 5 : pipe_max_chunk(s.N));
    int phase = dec ? e->phase : 0;  // decode-ahead: the games' step within their episode
    const unsigned nblk = (gpw == 32) ? (unsigned)((s.B + 32 * (kBlock / 64) - 1) / (32 * (kBlock / 64)))
                                      : (unsigned)grid_for(s.B);
    for (int t0 = 0; t0 < a.steps; t0 += chunk) {
        PlayArgs c = a;
        c.steps = min(chunk, a.steps - t0);
        c.step0 = a.step0 + t0;
        if (a.rewards) c.rewards = a.rewards + (int64_t)t0 * B * N;
        if (a.done) c.done = a.done + (int64_t)t0 * B;
        if (a.actions_out) c.actions_out = a.actions_out + (int64_t)t0 * B * N;
        if (a.obs) c.obs = a.obs + (int64_t)t0 * B * N * a.obs_stride;
        const uint64_t p = e->pphase;
        c.pipe_cin = (int)((p + kSlotMask) & kSlotMask), c.pipe_cout = (int)(p & kSlotMask);
        if (dec) {  // the launch's records: its episode's and (crossing a deal) the next one's
            c.n0 = phase;
            c.drec0 = (int)(e->dec_e % kDecRecords), c.drec1 = (int)((e->dec_e + 1) % kDecRecords);
        }
        const uint64_t G = p / (uint64_t)K;
        const bool first = (p % (uint64_t)K) == 0u;  // twist G beside this launch
        c.pipe_t = (int)((G + 1u) & 1u);              // twist G-1's end (INIT's for group 0)
        // twist G-1 (decode-ahead: decode G-1, which waited for twist G-1 itself)
        if (first && G >= 1u) HIP_TRY(hipStreamWaitEvent(st, (dec ? e->evd : e->evt)[(G + 1u) & 1u], 0));
        if (first && !e->pipe_serial) HIP_TRY(hipEventRecord(e->ev_main, st));  // launch p-1's consumption is final
        const int ti = (e->tn < e->tcap) ? e->tn++ : -1;  // SN_OPT_TIMING: this launch's events
        hipEvent_t* tv = (ti >= 0) ? e->tev + kTimingEvents * ti : nullptr;
        if (tv) e->tev_tw[ti] = first ? 1 : 0;
        if (tv) HIP_TRY(hipEventRecord(tv[0], st));
        {
            const sn_status r = dec ? dec_play(s, c, shmem, st) : pipe_play(s, c, gpw, nblk, shmem, st);
            if (r != SN_OK) return r;
        }
        const int64_t e_start = e->dec_e;  // the episode this launch started in
        if (dec) {
            phase += c.steps;
            if (phase >= kHand) phase -= kHand, e->dec_e++;
        }
        if (tv) HIP_TRY(hipEventRecord(tv[1], st));
        if (first) {
            // twist G, beside this launch (SECHS_PIPE_SERIAL=1, diagnostics: after it -- solo kernel times)
            if (e->pipe_serial) HIP_TRY(hipEventRecord(e->ev_main, st));
            HIP_TRY(hipStreamWaitEvent(e->side, e->ev_main, 0));
            if (tv) HIP_TRY(hipEventRecord(tv[2], e->side));
            // SN_OPT_TWIST_SKIP (tests only): the overrun detector under the default schedule
            const AheadArgs aa{dec ? kDecSlot + (int)((G + 1u) & 1u) : c.pipe_cin, c.pipe_t, (int)(G & 1u),
                               (e->twist_skip && G >= 1u) ? 0 : lead, e->perr_host_dev, -1};
            if (round_tw) hipLaunchKernelGGL((k_mt_ahead<false, true>), pg, dim3(kBlock), 0, e->side, s, aa);
            else hipLaunchKernelGGL((k_mt_ahead<false, false>), pg, dim3(kBlock), 0, e->side, s, aa);
            HIP_TRY(hipGetLastError());
            if (tv) HIP_TRY(hipEventRecord(tv[3], e->side));
            if (dec) {
                // decode G on side2, concurrent with twist G: the records group G+1 may touch --
                // its launches start at most K episodes past this launch's and touch at most one
                // more each: episodes < e_start + 2K + 1 (the ring of kDecRecords >= 2K + 2
                // slots never overwrites one a running launch reads: the oldest, launch p-K,
                // reads episodes >= e_start - K, 3K + 1 <= kDecRecords).  It reads the words twist
                // G-1 twisted (ptend slot (G-1) & 1) and waits for that twist only (which waited
                // for launch p-K-1), and its position goes to slot kDecSlot + (G & 1), which
                // twist G+1 reads.
                const int64_t target = e_start + 2 * K + 1;
                // (group 0: the start-up twist and decode ran on the play stream, before ev_main)
                if (e->pipe_serial || G == 0u) HIP_TRY(hipStreamWaitEvent(e->side2, e->ev_main, 0));
                if (G >= 1u) HIP_TRY(hipStreamWaitEvent(e->side2, e->evt[(G + 1u) & 1u], 0));
                if (tv) HIP_TRY(hipEventRecord(tv[4], e->side2));
                const int ne = target > e->dec_next ? (int)(target - e->dec_next) : 0;
                // ne == 0 (short launches): still a launch, so the position moves to slot G & 1
                const sn_status r = dec_launch(e, e->dec_next, ne, 0, (int)((G + 1u) & 1u),
                                               kDecSlot + (int)((G + 1u) & 1u), kDecSlot + (int)(G & 1u), e->side2);
                if (r != SN_OK) return r;
                e->dec_next = max(e->dec_next, target);
                if (tv) {
                    HIP_TRY(hipEventRecord(tv[5], e->side2));
                    e->tev_tw[ti] |= 2;
                }
                HIP_TRY(hipEventRecord(e->evd[G & 1u], e->side2));
            }
            HIP_TRY(hipEventRecord(e->evt[G & 1u], e->side));
            HIP_TRY(hipEventRecord(e->ev_prep, e->side));
            e->tw_out = (int)(G & 1u);
        }
        e->pl_cout = c.pipe_cout;
        e->pcount++;
        e->pphase++;
    }
    // behind this rollout's last k_play, on the caller's stream of THIS call:
    // the next call (or sn_pipe_sync) orders behind it without touching a
    // stream the caller may have destroyed since (one record per rollout)
    HIP_TRY(hipEventRecord(e->ev_play, st));
    return SN_OK;
}

static sn_status launch_play(sn_env* e, PlayArgs a, hipStream_t st) {
    const DevState& s = e->s;
    if (s.lg_K) {  // tournament handles: in-kernel DrunkHamster seats, pipelined numpy-MT or philox
        if (a.actions) return fail(SN_EUNSUPPORTED, "a tournament handle plays in-kernel DrunkHamster seats only (sn_rollout)");
        if (!(a.flags & SN_AUTO_RESET)) return fail(SN_EINVAL, "a tournament handle rolls out with SN_AUTO_RESET");
        if (s.rng_mode == SN_RNG_NUMPY_MT) {
            int wave;
            if (!e->pipe || e->pipe_gpw != 64 || pipe_lds(s, a, 64, &wave) > (size_t)kLdsBytes)
                return fail(SN_EUNSUPPORTED, "tournament rollouts need the pipelined numpy-MT path (64 games per wave)");
            return launch_pipe(e, a, st);
        }
        return launch_play_one(e, a, st);
    }
    if (s.rng_mode == SN_RNG_NUMPY_MT && !a.actions && e->pipe) {
        int wave;
        if (pipe_lds(s, a, e->pipe_gpw, &wave) <= (size_t)kLdsBytes) return launch_pipe(e, a, st);
    }
    {
        const sn_status r = sn_pipe_sync(e, st);
        if (r != SN_OK) return r;
    }
    const bool ring = (s.rng_mode == SN_RNG_NUMPY_MT) && !a.actions && s.ring_w > 0;
    if (!ring || a.steps <= e->chunk_steps) return launch_play_one(e, a, st);
    const int64_t B = s.B, N = s.N;
    for (int t0 = 0; t0 < a.steps; t0 += e->chunk_steps) {
        PlayArgs c = a;
        c.steps = min(e->chunk_steps, a.steps - t0);
        if (a.rewards) c.rewards = a.rewards + (int64_t)t0 * B * N;
        if (a.done) c.done = a.done + (int64_t)t0 * B;
        if (a.actions_out) c.actions_out = a.actions_out + (int64_t)t0 * B * N;
        if (a.obs) c.obs = a.obs + (int64_t)t0 * B * N * a.obs_stride;
        const sn_status r = launch_play_one(e, c, st);
        if (r != SN_OK) return r;
    }
    return SN_OK;
}

sn_status sn_step(sn_env* e, const int32_t* actions, int32_t* rewards, uint8_t* done, int32_t* invalid, int flags,
                  void* stream) {
    if (!e) return fail(SN_EINVAL, "env is NULL");
    if (e->s.lg_K) return fail(SN_EUNSUPPORTED, "a tournament handle plays whole games with sn_league_rollout");
    e->phase = -1;  // external actions may be refused per game
    PlayArgs a{};
    a.steps = 1;
    a.flags = flags;
    a.actions = actions;
    a.rewards = rewards;
    a.done = done;
    a.invalid = invalid;
    return launch_play(e, a, (hipStream_t)stream);
}

sn_status sn_rollout(sn_env* e, int steps, int32_t* rewards, uint8_t* done, uint8_t* actions, int8_t* obs,
                     int obs_stride, int flags, void* stream) {
    if (!e) return fail(SN_EINVAL, "env is NULL");
    if (steps < 0) return fail(SN_EINVAL, "steps must be >= 0");
    const int L = (flags & SN_NO_SUMMARIES) ? 35 : 47;
    if (obs && (obs_stride < L || (obs_stride & 3))) return fail(SN_EINVAL, "obs_stride must be a multiple of 4 and >= obs length");
    if (obs && (((uintptr_t)obs) & 3)) return fail(SN_EINVAL, "obs must be 4-byte aligned");
    if (steps == 0) return SN_OK;
    if (e->perr_host && __atomic_load_n(e->perr_host, __ATOMIC_RELAXED))
        return fail(SN_ERNG, "a pipelined numpy-MT draw ran past the twisted words; this handle's rollouts are invalid "
                             "from that launch on (sn_pipe_errors)");
    PlayArgs a{};
    a.steps = steps;
    a.flags = flags;
    a.obs_stride = obs_stride;
    a.rewards = rewards;
    a.done = done;
    a.actions_out = actions;
    a.obs = obs;
    const sn_status r = launch_play(e, a, (hipStream_t)stream);
    if (r == SN_OK && e->s.lg_K) e->lg_phase = (e->lg_phase + steps) % kHand;
    e->phase = (r == SN_OK && e->phase >= 0 && (flags & SN_AUTO_RESET)) ? (e->phase + steps) % kHand : -1;
    return r;
}

sn_status sn_league_config(sn_env* e, int num_agents, int min_players, int max_players) {
    if (!e) return fail(SN_EINVAL, "env is NULL");
    DevState& s = e->s;
    HIP_TRY(hipSetDevice(e->device));
    if (num_agents == 0) {
        HIP_TRY(hipDeviceSynchronize());
        if (s.lgs) (void)hipFree(s.lgs);
        s.lgs = nullptr;
        s.lg_K = s.lg_lo = s.lg_hi = 0;
        return SN_OK;
    }
    if (max_players != s.N) return fail(SN_EINVAL, "max_players must equal the handle's num_players");
    if (min_players < 2 || min_players > max_players || max_players > kLeagueMaxPlayers)
        return fail(SN_EINVAL, "need 2 <= min_players <= max_players <= 6");
    if (num_agents < max_players || num_agents > kLeagueMaxAgents)
        return fail(SN_EINVAL, "need max_players <= num_agents <= 16 (tournament.py:170 asserts len(self) >= num_players)");
    if (!s.lgs && hipMalloc((void**)&s.lgs, sizeof(uint32_t) * s.B) != hipSuccess) return fail(SN_ENOMEM, "league state");
    HIP_TRY(hipMemset(s.lgs, 0, sizeof(uint32_t) * s.B));
    s.lg_K = num_agents, s.lg_lo = min_players, s.lg_hi = max_players;
    for (int i = 0; i < kLeagueMaxAgents; i++) e->lg_kind[i] = SN_AGENT_RANDOM, e->lg_mpc[i] = 10, e->lg_mmax[i] = 100;
    e->lg_phase = -1;  // sn_reset deals the first games
    return SN_OK;
}

sn_status sn_league_rollout(sn_env* e, int steps, int32_t* rewards, uint8_t* done, uint8_t* actions, int8_t* obs,
                            int obs_stride, int32_t* records, void* stream) {
    if (!e) return fail(SN_EINVAL, "env is NULL");
    if (!e->s.lg_K) return fail(SN_EINVAL, "not a tournament handle (sn_league_config)");
    for (int i = 0; i < e->s.lg_K; i++)
        if (e->lg_kind[i] != SN_AGENT_RANDOM)
            return fail(SN_EUNSUPPORTED, "sn_league_rollout plays DrunkHamster agents in-kernel; mixed leagues use sn_league_step");
    if (e->lg_phase != 0) return fail(SN_EINVAL, "tournament rollouts start right after sn_reset or a whole number of games");
    if (steps % kHand) return fail(SN_EINVAL, "tournament rollouts play whole games (steps a multiple of 10)");
    if (steps < 0) return fail(SN_EINVAL, "steps must be >= 0");
    if (obs && (obs_stride < 47 || (obs_stride & 3))) return fail(SN_EINVAL, "obs_stride must be a multiple of 4 and >= 47");
    if (steps == 0) return SN_OK;
    if (e->perr_host && __atomic_load_n(e->perr_host, __ATOMIC_RELAXED))
        return fail(SN_ERNG, "a pipelined numpy-MT draw ran past the twisted words (sn_pipe_errors)");
    PlayArgs a{};
    a.steps = steps;
    a.flags = SN_AUTO_RESET;
    a.obs_stride = obs_stride;
    a.rewards = rewards;
    a.done = done;
    a.actions_out = actions;
    a.obs = obs;
    a.league_rec = records;
    return launch_play(e, a, (hipStream_t)stream);
}

// Host replay (no GPU): the reference scores a tournament game's Elo right
// after it (tournament.py:157-164), one game at a time; rl_6_nimmt/elo.py
// restates multi_elo's multiplayer Elo (parity unpinned).  Same operation
// order as elo.calc_elo, so the doubles match the Python replay bit for bit.
sn_status sn_elo_replay(const int32_t* rec, int64_t G, int NP, int K, double elo_k, double* elos) {
    if ((!rec && G > 0) || !elos) return fail(SN_EINVAL, "NULL argument");
    if (NP < 2 || NP > kLeagueMaxPlayers || K < 1 || K > kLeagueMaxAgents) return fail(SN_EINVAL, "bad sizes");
    for (int64_t i = 0; i < G; i++) {
        const int32_t* r = rec + i * (1 + NP);
        const uint32_t w = (uint32_t)r[0];
        const int k = (int)(w & 15u);
        if (k < 2 || k > NP) return fail(SN_EINVAL, "record " + std::to_string(i) + ": bad player count");
        int a[kLeagueMaxPlayers];
        double place[kLeagueMaxPlayers], old[kLeagueMaxPlayers], nw[kLeagueMaxPlayers];
        for (int p = 0; p < k; p++) {
            a[p] = (int)((w >> (4 + 4 * p)) & 15u);
            if (a[p] >= K) return fail(SN_EINVAL, "record " + std::to_string(i) + ": agent id out of range");
            old[p] = elos[a[p]];
        }
        for (int p = 0; p < k; p++) {  // Tournament._compute_absolute_positions: 1-based, ties averaged
            int greater = 0, equal = 0;
            for (int q = 0; q < k; q++) {
                greater += r[1 + q] > r[1 + p];
                equal += r[1 + q] == r[1 + p];
            }
            place[p] = (double)greater + 0.5 * (double)(1 + equal);
        }
        const double kk = elo_k / (double)(k - 1);
        for (int p = 0; p < k; p++) {
            double delta = 0.0;
            for (int q = 0; q < k; q++) {
                if (q == p) continue;
                const double actual = place[p] < place[q] ? 1.0 : (place[p] == place[q] ? 0.5 : 0.0);
                const double expected = 1.0 / (1.0 + std::pow(10.0, (old[q] - old[p]) / 400.0));
                delta += kk * (actual - expected);
            }
            nw[p] = old[p] + delta;
        }
        for (int p = 0; p < k; p++) elos[a[p]] = nw[p];
    }
    return SN_OK;
}

sn_status sn_league_seats(sn_env* e, uint32_t* out, void* stream) {
    if (!e || !out) return fail(SN_EINVAL, "NULL argument");
    if (!e->s.lg_K) return fail(SN_EINVAL, "not a tournament handle (sn_league_config)");
    HIP_TRY(hipMemcpyAsync(out, e->s.lgs, sizeof(uint32_t) * e->s.B, hipMemcpyDeviceToDevice, (hipStream_t)stream));
    return SN_OK;
}

sn_status sn_obs(sn_env* e, void* out, int dtype, int stride, int flags, void* stream) {
    if (!e || !out) return fail(SN_EINVAL, "NULL argument");
    const int L = (flags & SN_NO_SUMMARIES) ? 35 : 47;
    if (stride < L) return fail(SN_EINVAL, "obs stride shorter than the observation");
    const DevState& s = e->s;
    hipStream_t st = (hipStream_t)stream;
    const unsigned grid = grid_for(s.B * s.N);
    const int summ = !(flags & SN_NO_SUMMARIES);
    switch (dtype) {
        case SN_I8: hipLaunchKernelGGL(k_obs<int8_t>, dim3(grid), dim3(kBlock), 0, st, s, (int8_t*)out, stride, summ); break;
        case SN_I16: hipLaunchKernelGGL(k_obs<int16_t>, dim3(grid), dim3(kBlock), 0, st, s, (int16_t*)out, stride, summ); break;
        case SN_I32: hipLaunchKernelGGL(k_obs<int32_t>, dim3(grid), dim3(kBlock), 0, st, s, (int32_t*)out, stride, summ); break;
        case SN_I64: hipLaunchKernelGGL(k_obs<int64_t>, dim3(grid), dim3(kBlock), 0, st, s, (int64_t*)out, stride, summ); break;
        case SN_F32: hipLaunchKernelGGL(k_obs<float>, dim3(grid), dim3(kBlock), 0, st, s, (float*)out, stride, summ); break;
        default: return fail(SN_EINVAL, "unknown obs dtype");
    }
    HIP_TRY(hipGetLastError());
    return SN_OK;
}

sn_status sn_hands(sn_env* e, int8_t* out, void* stream) {
    if (!e || !out) return fail(SN_EINVAL, "NULL argument");
    hipLaunchKernelGGL(k_hands, dim3(grid_for(e->s.B * e->s.N)), dim3(kBlock), 0, (hipStream_t)stream, e->s, out);
    HIP_TRY(hipGetLastError());
    return SN_OK;
}

sn_status sn_board(sn_env* e, int8_t* out, void* stream) {
    if (!e || !out) return fail(SN_EINVAL, "NULL argument");
    hipLaunchKernelGGL(k_board, dim3(grid_for(e->s.B)), dim3(kBlock), 0, (hipStream_t)stream, e->s, out);
    HIP_TRY(hipGetLastError());
    return SN_OK;
}

sn_status sn_scores(sn_env* e, int32_t* out, void* stream) {
    if (!e || !out) return fail(SN_EINVAL, "NULL argument");
    hipLaunchKernelGGL(k_scores, dim3(grid_for(e->s.B)), dim3(kBlock), 0, (hipStream_t)stream, e->s, out,
                       (int32_t*)nullptr, (int32_t*)nullptr);
    HIP_TRY(hipGetLastError());
    return SN_OK;
}

sn_status sn_results(sn_env* e, int32_t* sum_results, int32_t* episodes, void* stream) {
    if (!e) return fail(SN_EINVAL, "NULL argument");
    hipLaunchKernelGGL(k_scores, dim3(grid_for(e->s.B)), dim3(kBlock), 0, (hipStream_t)stream, e->s,
                       (int32_t*)nullptr, sum_results, episodes);
    HIP_TRY(hipGetLastError());
    return SN_OK;
}

sn_status sn_clear_results(sn_env* e, void* stream) {
    if (!e) return fail(SN_EINVAL, "NULL argument");
    hipLaunchKernelGGL(k_clear_results, dim3(grid_for(e->s.B)), dim3(kBlock), 0, (hipStream_t)stream, e->s);
    HIP_TRY(hipGetLastError());
    return SN_OK;
}

// lazy -> numpy form: finish the current round for words [p, 624)
static void mt_finish_round(uint32_t* a, int p) {
    for (int i = p; i < kMtN; i++) {
        uint32_t y = (a[i] & 0x80000000u) | (a[(i + 1) % kMtN] & 0x7fffffffu);
        a[i] = a[(i + kMtM) % kMtN] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
    }
}

// Undo the twist of the new round's words [0, T): new[j] = src ^ (y >> 1) ^
// (y & 1 ? A : 0) with y = (old[j] & UPPER) | (old[j+1] & LOWER) and src =
// new[j-227] (j >= 227) or old[j+397] (j < 227: still in place, or itself
// restored from the j >= 227 words when T > 397).  A's top bit is set and
// y >> 1's is not, so the top bit of new[j] ^ src is y & 1 and y follows.
// old[0]'s low 31 bits never enter the twist; they come from mt0.
static uint32_t mt_untwist_y(uint32_t t) {
    const uint32_t lsb = t >> 31;
    if (lsb) t ^= 0x9908b0dfu;
    return (t << 1) | lsb;
}

static void mt_unstraddle(uint32_t* a, int T, uint32_t old0) {
    constexpr int D = kMtN - kMtM;  // 227
    uint32_t y[kMtN];
    for (int j = D; j < T; j++) y[j] = mt_untwist_y(a[j] ^ a[j - D]);
    auto old_at = [&](int m) -> uint32_t {  // m >= 397
        return (m < T) ? ((y[m] & 0x80000000u) | (y[m - 1] & 0x7fffffffu)) : a[m];
    };
    for (int j = 0; j < T && j < D; j++) y[j] = mt_untwist_y(a[j] ^ old_at(j + kMtM));
    for (int j = 0; j < T; j++) a[j] = (y[j] & 0x80000000u) | ((j == 0 ? old0 : y[j - 1]) & 0x7fffffffu);
}

sn_status sn_mt_get(sn_env* e, int64_t game, uint32_t* key, int32_t* pos) {
    if (!e || !key || !pos) return fail(SN_EINVAL, "NULL argument");
    if (e->s.rng_mode != SN_RNG_NUMPY_MT) return fail(SN_EINVAL, "env is not in numpy-compat RNG mode");
    if (game < 0 || game >= e->s.B) return fail(SN_EINVAL, "game out of range");
    HIP_TRY(hipSetDevice(e->device));
    if (sn_pipe_sync(e, 0) != SN_OK) return SN_EHIP;
    HIP_TRY(hipDeviceSynchronize());
    uint32_t code = 0;
    HIP_TRY(hipMemcpy(key, e->s.mt + game * kMtN, sizeof(uint32_t) * kMtN, hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(&code, e->s.mt_pos + game, sizeof(uint32_t), hipMemcpyDeviceToHost));
    // decode (sechs_device.h MtGenT): words [pos-cnt, pos) twisted, unconsumed
    const int p = (int)(code & 0x7FFu), cnt = (int)((code >> 16) & kMtCntMask);
    if (cnt > p && p > 0) {  // straddling: still in the previous round, whose head [0, p) was overwritten
        uint32_t old0 = 0;
        HIP_TRY(hipMemcpy(&old0, e->s.mt0 + game, sizeof(uint32_t), hipMemcpyDeviceToHost));
        mt_unstraddle(key, p, old0);
    } else if (p > 0 && p < kMtN) {
        mt_finish_round(key, p);  // twist the rest of this round in place
    }
    *pos = (int32_t)mt_numpy_pos(code);
    return SN_OK;
}

sn_status sn_mt_set(sn_env* e, int64_t game, const uint32_t* key, int32_t pos) {
    if (!e || !key) return fail(SN_EINVAL, "NULL argument");
    if (e->s.rng_mode != SN_RNG_NUMPY_MT) return fail(SN_EINVAL, "env is not in numpy-compat RNG mode");
    if (game < 0 || game >= e->s.B) return fail(SN_EINVAL, "game out of range");
    if (pos < 0 || pos > kMtN) return fail(SN_EINVAL, "pos must be in 0..624");
    HIP_TRY(hipSetDevice(e->device));
    if (sn_pipe_sync(e, 0) != SN_OK) return SN_EHIP;
    HIP_TRY(hipDeviceSynchronize());
    const uint32_t code = mt_code_from_numpy(pos);
    HIP_TRY(hipMemcpy(e->s.mt + game * kMtN, key, sizeof(uint32_t) * kMtN, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(e->s.mt_pos + game, &code, sizeof(uint32_t), hipMemcpyHostToDevice));
    return SN_OK;
}

static sn_status h1_ready(sn_env* e) {
    if (e->s.B != 1) return fail(SN_EINVAL, "the one-game fast path needs a one-game handle");
    if (!e->hbuf) {
        if (hipHostMalloc((void**)&e->hbuf, sizeof(uint32_t) * kH1Words, hipHostMallocMapped) != hipSuccess ||
            hipHostGetDevicePointer((void**)&e->hbuf_dev, e->hbuf, 0) != hipSuccess)
            return fail(SN_ENOMEM, "pinned exchange buffer");
    }
    return SN_OK;
}

// out_host: the 2 + 14 N result words, then N trace words (sn_step1; zeros for a reset)
static void h1_copy_out(const sn_env* e, int32_t* out, bool trace) {
    const int N = e->s.N;
    std::memcpy(out, e->hbuf + kH1Out, sizeof(uint32_t) * (2 + 2 * N + 12 * N));
    if (trace) std::memcpy(out + 2 + 14 * N, e->hbuf + kH1Out + kH1Trace, sizeof(uint32_t) * N);
    else std::memset(out + 2 + 14 * N, 0, sizeof(uint32_t) * N);
}

sn_status sn_step1(sn_env* e, const int32_t* actions_host, int32_t* out_host, int flags) {
    if (!e || !actions_host || !out_host) return fail(SN_EINVAL, "NULL argument");
    HIP_TRY(hipSetDevice(e->device));
    if (h1_ready(e) != SN_OK) return SN_ENOMEM;
    if (e->s.lg_K) return fail(SN_EUNSUPPORTED, "a tournament handle plays whole games with sn_league_rollout");
    e->phase = -1;
    Acts1 a{};
    for (int p = 0; p < e->s.N; p++) a.a[p] = actions_host[p];
    const int summ = !(flags & SN_NO_SUMMARIES);
    SN_DISPATCH_N(e->s.N, hipLaunchKernelGGL((k_step1<NN>), dim3(1), dim3(64), 0, 0, e->s, a, e->hbuf_dev, summ));
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipStreamSynchronize(0));
    h1_copy_out(e, out_host, true);
    return SN_OK;
}

sn_status sn_reset1(sn_env* e, const uint32_t* key_host, int32_t pos, uint32_t* key_out_host, int32_t* pos_out,
                    int32_t* out_host, int flags) {
    if (!e || !key_host || !key_out_host || !pos_out || !out_host) return fail(SN_EINVAL, "NULL argument");
    if (e->s.rng_mode != SN_RNG_NUMPY_MT) return fail(SN_EINVAL, "env is not in numpy-compat RNG mode");
    if (pos < 0 || pos > kMtN) return fail(SN_EINVAL, "pos must be in 0..624");
    HIP_TRY(hipSetDevice(e->device));
    if (h1_ready(e) != SN_OK) return SN_ENOMEM;
    if (e->s.lg_K) return fail(SN_EUNSUPPORTED, "a tournament handle deals with sn_reset");
    if (sn_pipe_sync(e, 0) != SN_OK) return SN_EHIP;
    std::memcpy(e->hbuf + kH1In, key_host, sizeof(uint32_t) * kMtN);
    e->hbuf[kH1In + kMtN] = (uint32_t)pos;
    const int summ = !(flags & SN_NO_SUMMARIES);
    SN_DISPATCH_N(e->s.N, hipLaunchKernelGGL((k_reset1<NN>), dim3(1), dim3(64), 0, 0, e->s, e->hbuf_dev, summ));
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipStreamSynchronize(0));
    e->phase = 0;  // one game, just dealt
    h1_copy_out(e, out_host, false);
    // the advanced state in numpy's (key, pos) form, as sn_mt_get
    std::memcpy(key_out_host, e->hbuf + kH1Mt, sizeof(uint32_t) * kMtN);
    const uint32_t code = e->hbuf[kH1Mt + kMtN];
    const int p = (int)(code & 0x7FFu), cnt = (int)((code >> 16) & kMtCntMask);
    if (cnt > p && p > 0) mt_unstraddle(key_out_host, p, e->hbuf[kH1Mt + kMtN + 1]);
    else if (p > 0 && p < kMtN) mt_finish_round(key_out_host, p);
    *pos_out = (int32_t)mt_numpy_pos(code);
    return SN_OK;
}

sn_status sn_kernel_times(sn_env* e, float* play_ms, float* ahead_ms, int32_t* n) {
    return sn_kernel_times_dec(e, play_ms, ahead_ms, nullptr, n);
}

sn_status sn_kernel_times_dec(sn_env* e, float* play_ms, float* ahead_ms, float* decode_ms, int32_t* n) {
    if (!e || !play_ms || !ahead_ms || !n) return fail(SN_EINVAL, "NULL argument");
    HIP_TRY(hipSetDevice(e->device));
    HIP_TRY(hipDeviceSynchronize());
    double sp = 0.0, sa = 0.0, sd = 0.0;
    int na = 0, nd = 0;
    for (int i = 0; i < e->tn; i++) {
        const hipEvent_t* tv = e->tev + kTimingEvents * i;
        float a = 0.f, b = 0.f, c = 0.f;
        HIP_TRY(hipEventElapsedTime(&a, tv[0], tv[1]));
        sp += a;
        if (e->tev_tw[i] & 1) {  // a twist ran beside this launch (the first of its group)
            HIP_TRY(hipEventElapsedTime(&b, tv[2], tv[3]));
            sa += b, na++;
        }
        if (e->tev_tw[i] & 2) {  // and a decode-ahead launch after it
            HIP_TRY(hipEventElapsedTime(&c, tv[4], tv[5]));
            sd += c, nd++;
        }
    }
    *n = e->tn;
    *play_ms = e->tn ? (float)(sp / e->tn) : 0.f;
    *ahead_ms = na ? (float)(sa / na) : 0.f;
    if (decode_ms) *decode_ms = nd ? (float)(sd / nd) : 0.f;
    return SN_OK;
}

sn_status sn_debug_phases(uint64_t* out, int n) {
    if (!out || n < 1) return fail(SN_EINVAL, "NULL argument");
#ifdef SECHS_PHASE_PROF
    unsigned long long h[PH_N + 2];
    HIP_TRY(hipDeviceSynchronize());
    HIP_TRY(hipMemcpyFromSymbol(h, HIP_SYMBOL(g_phase), sizeof(h)));
    for (int k = 0; k < n; k++) out[k] = (k <= PH_N + 1) ? (uint64_t)h[k] : 0ull;
    const unsigned long long z[PH_N + 2] = {};
    HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(g_phase), z, sizeof(z)));
    return SN_OK;
#else
    for (int k = 0; k < n; k++) out[k] = 0ull;
    return fail(SN_EUNSUPPORTED, "built without SECHS_PHASE_PROF (make libsechs_prof.so)");
#endif
}

#if defined(SECHS_DEBUG)
__global__ void k_debug_selftest(int fail) { SN_DASSERT(fail == 0); }
#endif

sn_status sn_debug_failures(uint32_t* count, uint32_t* first_line, int selftest) {
    if (!count || !first_line) return fail(SN_EINVAL, "NULL argument");
    *count = 0u, *first_line = 0u;
#if defined(SECHS_DEBUG)
    if (selftest) {  // one deliberately violated assertion: proves the counter is live
        hipLaunchKernelGGL(k_debug_selftest, dim3(1), dim3(1), 0, 0, 1);
        HIP_TRY(hipGetLastError());
    }
    unsigned int h[2];
    HIP_TRY(hipDeviceSynchronize());
    HIP_TRY(hipMemcpyFromSymbol(h, HIP_SYMBOL(g_sn_dbg), sizeof(h)));
    *count = h[0], *first_line = h[1];
    const unsigned int z[2] = {0u, 0xFFFFFFFFu};
    HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(g_sn_dbg), z, sizeof(z)));
    return SN_OK;
#else
    (void)selftest;
    return fail(SN_EUNSUPPORTED, "built without SECHS_DEBUG (make libsechs_debug.so)");
#endif
}

sn_status sn_pipe_errors(sn_env* e, uint32_t* count) {
    if (!e || !count) return fail(SN_EINVAL, "NULL argument");
    *count = 0;
    if (!e->s.perr) return SN_OK;
    HIP_TRY(hipSetDevice(e->device));
    HIP_TRY(hipDeviceSynchronize());
    HIP_TRY(hipMemcpy(count, e->s.perr, sizeof(uint32_t), hipMemcpyDeviceToHost));
    if (e->perr_host && *count) __atomic_store_n(e->perr_host, *count, __ATOMIC_RELAXED);
    return SN_OK;
}

sn_status sn_debug_pipe_words(sn_env* e, int what, int slot, uint32_t* out) {
    if (!e || !out) return fail(SN_EINVAL, "NULL argument");
    if (!e->s.pabsc) return fail(SN_EUNSUPPORTED, "no pipeline (numpy-compat handles only)");
    const int64_t B = e->s.B;
    const void* src = nullptr;
    size_t bytes = 0;
    if (what == 0 && slot >= 0 && slot <= kPipeSlots) src = e->s.pabsc + (int64_t)slot * B, bytes = 4 * B;
    else if (what == 1 && slot >= 0 && slot < 2) src = e->s.ptend + (int64_t)slot * B, bytes = 4 * B;
    else if (what == 2 && slot >= 0 && slot < kDecRecords && e->s.drec)
        src = e->s.drec + (int64_t)slot * kDecQuads * B, bytes = sizeof(u32x4) * kDecQuads * B;
    else return fail(SN_EINVAL, "what / slot out of range");
    HIP_TRY(hipSetDevice(e->device));
    HIP_TRY(hipDeviceSynchronize());
    HIP_TRY(hipMemcpy(out, src, bytes, hipMemcpyDeviceToHost));
    return SN_OK;
}

sn_status sn_philox_counter(sn_env* e, int64_t game, uint64_t* ctr) {
    if (!e || !ctr) return fail(SN_EINVAL, "NULL argument");
    if (game < 0 || game >= e->s.B) return fail(SN_EINVAL, "game out of range");
    HIP_TRY(hipSetDevice(e->device));
    HIP_TRY(hipDeviceSynchronize());
    HIP_TRY(hipMemcpy(ctr, e->s.ctr + game, sizeof(uint64_t), hipMemcpyDeviceToHost));
    return SN_OK;
}

}  // extern "C"

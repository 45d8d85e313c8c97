// sechs_quad.h -- the headline rollout with four lanes per game (k_play_quad).
//
// Included by sechs_env.hip after PlayArgs / PhaseProf / st_nt.  Same
// contract as k_play<4, RNG_NUMPY_PIPE> (in-kernel DrunkHamster seats,
// pipelined numpy-MT ring, optional int8 obs rows of 48 bytes, rewards,
// actions, done, auto-reset) and the same words consumed in the same order,
// so its outputs are bit-identical; what changes is the mapping.  k_play
// gives each game one lane: at B = 65 536 that is 1 024 waves, one per
// SIMD, and a lone wave issues at most one VALU every 4 cycles and hides
// none of its LDS / memory latency.  Here a game is a quad of
// lanes (16 games per wave, 4 096 waves, four per SIMD), and lane q of the
// quad is seat q AND board row q:
//   * seat work is the lane's own: its hand, its DrunkHamster draw (the
//     (q+1)-th accepted word of the step's window, agents/random.py:9 in
//     seat order, play.py:38-41), its observation row (env.py:188-212), its
//     reward / action / score / result, its sorted hand after a deal;
//   * row work is the lane's own too: _find_row / _pick_row_to_replace
//     (env.py:138-160) become two quad reductions over the lanes' rows
//     (max of the rows ending below the card, min of the row heads) and only
//     the target row's lane updates it (env.py:127-134, _score_row 162-172);
//   * the game's shared state (hand size, stream position) is replicated in
//     the four lanes, computed identically from the same data.
// Cross-lane traffic is DPP quad permutes (no LDS).  The deal's Fisher-Yates
// swaps (env.py:99-112, numpy's shuffle) run one LDS round trip per word:
// few instructions per word, and with four waves per SIMD the round trips of
// one wave overlap the others' work.
#pragma once

namespace sechs {

constexpr int kQuadGames = 16;   // games per wave
constexpr int kQuadStage = 192;  // LDS bytes per game: 4 obs rows x 48 (lane-major); the wave's area doubles as decks
constexpr int kQuadDeck = 108;   // the deal's deck per game inside that area: 27 dwords, an odd stride, so the
                                 // 16 games' deck[i] (the same i in lockstep) fall in 16 distinct banks
constexpr int kQuadSlot = 272;   // LDS bytes per game: the RingPipe window (16 chunks + the funnel's 8, 16-aligned)
constexpr int kQuadRound = kMtN * 4;  // SN_OPT_PIPE_FUSED: one MT19937 round (the wave's round buffer, LDS-DMA target)
constexpr int kQuadWave = kQuadGames * (kQuadStage + kQuadSlot) + kQuadRound;  // 9 920 B: 4 blocks of 4 waves per CU
static_assert(kQuadSlot >= ((kPipeWin + 15 + 15) / 16) * 16 + 16, "window + funnel reads");
static_assert(kQuadDeck >= kMaxCards && kQuadGames * kQuadDeck <= kQuadGames * kQuadStage, "decks fit the staging area");

// lane k of this lane's quad (DPP quad_perm, no LDS)
template <int K>
__device__ __forceinline__ uint32_t qget(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, K * 0x55, 0xF, 0xF, false);
}
__device__ __forceinline__ uint32_t qmax(uint32_t v) {
    v = max(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false));  // [1,0,3,2]
    return max(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, false));  // [2,3,0,1]
}
__device__ __forceinline__ uint32_t qmin(uint32_t v) {
    v = min(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false));
    return min(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, false));
}

// acceptance bytes (0x80 / 0x00, swar_le_mask) of 8 words -> 8 bits
__device__ __forceinline__ uint32_t acc_bits8(uint64_t a) {
    // bit 8i+7 of a dword lands at bit 28+i of d * 0x00204081; the cross
    // terms stay below bit 24 (no carry reaches bit 28)
    const uint32_t lo = ((uint32_t)a * 0x00204081u) >> 28;
    const uint32_t hi = ((uint32_t)(a >> 32) * 0x00204081u) >> 28;
    return lo | (hi << 4);
}

// Past the LDS window (rare): bytes of stream positions pos.. from the HBM
// ring; positions at or past the twisted end read as 0 (the launch then
// consumed more than `avail` and counts an error at its end).
static __device__ __noinline__ uint64_t quad_slow8(const uint8_t* ring, int64_t B, int64_t g, uint32_t pos,
                                                   uint32_t left) {
    uint64_t r = 0ull;
    const uint32_t k = min(8u, left);
    for (uint32_t i = 0; i < k; i++) {
        const uint32_t ri = (pos + i) & (uint32_t)(kPipeRing - 1);
        r |= (uint64_t)ring[ring_byte(ri, g, B)] << (8u * i);
    }
    return r;
}

// The game's pipelined word stream, by position t relative to the launch's
// consumer position c0 (replicated in the quad: no byte buffer, every read
// is by position from the LDS window).
struct QuadPipe {
    const uint8_t* slot;
    const uint8_t* ring;
    int64_t B, g;
    uint32_t c0, avail, win, off;

    __device__ __forceinline__ void load(const DevState& s, int64_t gg, int q, uint8_t* lds_slot, int cin, int tpar,
                                         bool& bad) {
        g = gg, B = s.B;
        c0 = s.pabsc[(int64_t)cin * B + g];
        const int32_t av = (int32_t)(s.ptend[(int64_t)tpar * B + g] - c0);
        bad = av < 0;
        avail = bad ? 0u : (uint32_t)av;
        win = min(avail, (uint32_t)kPipeWin);
        off = c0 & 15u;
        slot = lds_slot;
        ring = (const uint8_t*)s.pring;
        const uint32_t q0 = (c0 & (uint32_t)(kPipeRing - 1)) >> 4;
        const uint32_t nch = (off + win + 15u) >> 4;
        for (uint32_t i = (uint32_t)q; i < nch; i += 4u)  // the quad copies its window 4 chunks at a time
            *(u32x4*)(lds_slot + 16u * i) = s.pring[ring16(q0 + i, g, B)];
    }
    // bytes t .. t+7
    __device__ __forceinline__ uint64_t peek8(uint32_t t) const {
        if (t + 8u <= win) {
            const uint32_t p = off + t, a8 = p & ~7u, sh = 8u * (p & 7u);
            const uint64_t lo = *(const uint64_t*)(slot + a8);
            const uint64_t hi = *(const uint64_t*)(slot + a8 + 8u);
            return sh ? ((lo >> sh) | (hi << (64u - sh))) : lo;
        }
        return quad_slow8(ring, B, g, c0 + t, (avail > t) ? avail - t : 0u);
    }
    // bytes t .. t+15 (three aligned reads on the fast path)
    __device__ __forceinline__ void peek16(uint32_t t, uint64_t& w0, uint64_t& w1) const {
        if (t + 16u <= win) {
            const uint32_t p = off + t, a8 = p & ~7u, sh = 8u * (p & 7u);
            const uint64_t x0 = *(const uint64_t*)(slot + a8);
            const uint64_t x1 = *(const uint64_t*)(slot + a8 + 8u);
            const uint64_t x2 = *(const uint64_t*)(slot + a8 + 16u);
            w0 = sh ? ((x0 >> sh) | (x1 << (64u - sh))) : x0;
            w1 = sh ? ((x1 >> sh) | (x2 << (64u - sh))) : x1;
            return;
        }
        w0 = peek8(t);
        w1 = peek8(t + 8u);
    }
};

// One step's DrunkHamster draws for the 4 seats (all with max = n - 1):
// seat q takes the (q+1)-th accepted word from position t; the quad
// advances t past the 4th.  Returns this lane's masked value.
__device__ __forceinline__ uint32_t quad_draw(const QuadPipe& P, uint32_t& t, uint32_t max, int q) {
    if (max == 0u) return 0u;  // numpy: random_interval(0) draws nothing
    const uint32_t mask = 0xFFFFFFFFu >> __builtin_clz(max);
    const uint64_t mb = 0x0101010101010101ull * (uint64_t)mask;
    uint32_t got = 0u, v = 0u;
    while (true) {  // quad-uniform: every lane sees the same window
        uint64_t w0, w1;
        P.peek16(t, w0, w1);
        const uint64_t x0 = w0 & mb, x1 = w1 & mb;
        const uint32_t m16 = acc_bits8(swar_le_mask(x0, max)) | (acc_bits8(swar_le_mask(x1, max)) << 8);
        const uint32_t cnt = __popc(m16);
        // this lane's accept is number k = q - got of the window
        const uint32_t k = (uint32_t)q - got;
        uint32_t m = m16;
        m = (k > 0u) ? (m & (m - 1u)) : m;
        m = (k > 1u) ? (m & (m - 1u)) : m;
        m = (k > 2u) ? (m & (m - 1u)) : m;
        const uint32_t pos = __builtin_ctz(m | 0x10000u);  // byte index of this lane's accept (16: not here)
        const uint32_t val = (uint32_t)(((pos < 8u) ? x0 : x1) >> (8u * (pos & 7u))) & 0xFFu;
        if ((uint32_t)q >= got && k < cnt) v = val;
        if (got + cnt >= 4u) {
            t += qget<3>(pos) + 1u;  // through seat 3's word
            return v;
        }
        got += cnt;
        t += 16u;
    }
}

// place card c (heads hc) on the quad's board, env.py:127-134: returns the
// bull heads its player takes (quad-uniform); lane q's row is (rlo, rhi)
__device__ __forceinline__ uint32_t quad_place(uint32_t& rlo, uint32_t& rhi, uint32_t c, uint32_t hc, int q) {
    const uint32_t e = end_of(rhi), len = len_of(rhi), hd = heads_in(rhi);
    // _find_row: the largest row end below c -- (end + 1, row, heads, len) of it
    const uint32_t cand = (e < c) ? (((e + 1u) << 16) | ((uint32_t)q << 12) | (hd << 4) | len) : 0u;
    const uint32_t best = qmax(cand);
    // _pick_row_to_replace: np.argmin of the row heads, first minimum
    const uint32_t mn = qmin((hd << 2) | (uint32_t)q);
    const bool under = best == 0u;
    const uint32_t tr = under ? (mn & 3u) : ((best >> 12) & 3u);
    const bool take = under || (best & 15u) == (uint32_t)(kThreshold - 1);  // the 6th card
    const uint32_t pen = take ? (under ? (mn >> 2) : ((best >> 4) & 0xFFu)) : 0u;  // _score_row: the old row
    SN_DASSERT(under || (best >> 16) - 1u < c);                       // the target row ends below the card
    SN_DASSERT(len >= 1u && len <= (uint32_t)(kThreshold - 1));        // every row holds 1..5 cards
    // only the target row's lane changes its row (selects, no branch)
    const uint32_t lo_n = take ? c : (rlo | (len < 4u ? (c << (8u * len)) : 0u));
    const uint32_t hi_n = take ? ((1u << 8) | (hc << 16) | (c << 24))
                               : ((len == 4u ? c : (rhi & 0xFFu)) | ((len + 1u) << 8) | ((hd + hc) << 16) | (c << 24));
    const bool mine = (uint32_t)q == tr;
    rlo = mine ? lo_n : rlo;
    rhi = mine ? hi_n : rhi;
    return pen;
}

// The round's old words by LDS-DMA (global_load_lds_dwordx4, 1 KiB per
// wave instruction, no VGPRs): three instructions for the 2 496 bytes.
// Issued as inline asm, so hipcc neither counts them nor makes the step
// loop's other LDS accesses wait for them (every LDS access of this kernel
// may alias the one dynamic array); the consumer waits with an explicit
// `s_waitcnt vmcnt(0)` a whole env-step later.
__device__ __forceinline__ void glds16(const void* gsrc, uint32_t lds_dst) {
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(gsrc), "s"(lds_dst)
                 : "memory");
}
__device__ __forceinline__ void quad_round_issue(const DevState& s, int64_t G, uint32_t lane, uint32_t* w) {
    const uint8_t* src = (const uint8_t*)(s.mt + G * kMtN) + 16u * lane;
    const uint32_t dst = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(uintptr_t)w);  // LDS byte address
    glds16(src, dst);
    glds16(src + 1024, dst + 1024u);
    if (lane < (uint32_t)(kMtN * 4 - 2048) / 16u) glds16(src + 2048, dst + 2048u);
}
__device__ __forceinline__ void vm_drain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// compare-exchange of two sort keys
__device__ __forceinline__ void qce(uint32_t& a, uint32_t& b) {
    const uint32_t lo = min(a, b), hi = max(a, b);
    a = lo, b = hi;
}

__global__ __launch_bounds__(kBlock, 4) void k_play_quad(DevState s, PlayArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds_dyn[];
    const int tid = (int)threadIdx.x, lane = tid & 63, q = lane & 3, gl = lane >> 2;
    const int64_t B = s.B;
    const int64_t g0 = ((int64_t)blockIdx.x * (kBlock / 64) + (tid >> 6)) * kQuadGames;  // first game of the wave
    const int64_t g = g0 + gl;
    if (g >= B) return;  // whole quads
    const int wave_games = (int)min((int64_t)kQuadGames, B - g0);
    __builtin_amdgcn_s_setprio(1);  // over co-resident k_mt_ahead waves, as k_play
    uint8_t* wl = lds_dyn + (tid >> 6) * kQuadWave;
    u32x4* stage = (u32x4*)wl;  // the wave's obs rows, lane-major (3 pieces per lane: an odd stride)
    uint8_t* deck = wl + gl * kQuadDeck;  // (staging is idle during a deal: same wave, program order)
    PhaseProf pp;
    pp.start();
    // ---- load: seat q's hand / score / results, row q, the stream window
    Hand h;
    {
        const uint32_t w0 = s.hand[(int64_t)(q * 3 + 0) * B + g];
        const uint32_t w1 = s.hand[(int64_t)(q * 3 + 1) * B + g];
        h.lo = (uint64_t)w0 | ((uint64_t)w1 << 32);
        h.hi = s.hand[(int64_t)(q * 3 + 2) * B + g];
    }
    uint32_t rlo = s.row_lo[(int64_t)q * B + g], rhi = s.row_hi[(int64_t)q * B + g];
    int32_t score = s.score[(int64_t)q * B + g];
    const bool auto_reset = (a.flags & SN_AUTO_RESET) != 0;
    const bool summ = !(a.flags & SN_NO_SUMMARIES);
    int32_t sres = 0, eps = 0;
    if (auto_reset) {
        sres = s.sum_res[(int64_t)q * B + g];
        eps = s.episodes[g];
    }
    uint32_t n = hand_len(h);  // every seat holds the same count
    QuadPipe P;
    bool bad_start;
    P.load(s, g, q, wl + kQuadGames * kQuadStage + gl * kQuadSlot, a.pipe_cin, a.pipe_t, bad_start);
    uint32_t t = 0u;
    // SN_OPT_PIPE_FUSED: the games of this wave whose twisted lead is short get
    // their next round twisted by this launch, one per env-step: the round's
    // words are LDS-DMA'd into the wave's round buffer at the step's start and
    // twisted at its end, so the load's latency hides behind the step (a
    // register-staged round would hold 10 VGPRs across the step).  Rounds
    // past the steps (more needy games than steps, rare) run after the loop.
    // The words are for the NEXT launches -- this one reads below the
    // twisted end it started with (P.avail) -- and the ring holds lead + 624
    // < kPipeRing words.
    const bool fused = a.fuse_lead > 0;
    uint32_t twisted = 0u;  // this game's round was twisted (quad-uniform)
    uint32_t te0 = 0u, my_old0 = 0u;
    uint64_t tw_todo = 0ull;  // needy games (bit 4 gl), not yet issued
    int tw_fly = -1;          // the bit of the game whose round is in the buffer / in flight
    uint32_t* rbuf = (uint32_t*)(wl + kQuadGames * (kQuadStage + kQuadSlot));
    if (fused) {
        if (blockIdx.x == 0 && tid == 0 && a.perr_mirror)  // overruns so far (earlier launches), as k_mt_ahead does
            __hip_atomic_store(a.perr_mirror, __hip_atomic_load(s.perr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        te0 = s.ptend[(int64_t)a.pipe_t * B + g];
        const uint32_t Tp = s.ptp[g];
        // not round-aligned (the fused start completes rounds, so never): an error, no twist
        const bool need = q == 0 && !bad_start && P.avail < (uint32_t)a.fuse_lead;
        if (need && Tp != (uint32_t)kMtN) atomicAdd(s.perr, 1u);
        tw_todo = __ballot(need && Tp == (uint32_t)kMtN);
    }
    // issue the next needy game's round into the buffer (wave-uniform)
    if (a.dbg & 8) tw_todo = 0ull;  // timing diagnostics only (SECHS_QUAD_DBG bit 3: no twist; overruns follow)
    auto tw_issue = [&]() {
        if (tw_fly < 0 && tw_todo) {
            tw_fly = (int)__builtin_ctzll(tw_todo);
            tw_todo &= tw_todo - 1ull;
            quad_round_issue(s, g0 + (tw_fly >> 2), (uint32_t)lane, rbuf);
        }
    };
    // twist the round in the buffer (waits for its DMA and everything before it)
    auto tw_finish = [&]() {
        if (tw_fly >= 0) {
            vm_drain();
            const int64_t G = g0 + (tw_fly >> 2);
            const uint32_t teG = (uint32_t)__builtin_amdgcn_readlane((int)te0, tw_fly);
            // (SECHS_QUAD_DBG bit 4, timing diagnostics only: the DMA and its wait, no twist)
            const uint32_t old0 = (a.dbg & 16) ? 0u : mt_twist_round(s, G, (uint32_t)lane, rbuf, teG);
            if (lane == tw_fly) my_old0 = old0;
            if (gl == (tw_fly >> 2)) twisted = 1u;
            tw_fly = -1;
        }
    };
    pp.mark(PH_PROLOGUE);
    const int C = s.C;
    for (int step = 0; step < a.steps; step++) {
        if (fused) tw_issue();
        // ---- observation rows (pre-action), env.py:174-212
        if (a.obs) {
            Board b;
            b.lo = u32x4{qget<0>(rlo), qget<1>(rlo), qget<2>(rlo), qget<3>(rlo)};
            b.hi = u32x4{qget<0>(rhi), qget<1>(rhi), qget<2>(rhi), qget<3>(rhi)};
            uint32_t w2hi;
            const GameWords gw = summ ? game_words<true>(4, b, w2hi) : game_words<false>(4, b, w2hi);
            u32x4* row = stage + 3 * lane;
            row[0] = u32x4{(uint32_t)h.lo, (uint32_t)(h.lo >> 32), (h.hi & 0xFFFFu) | w2hi, gw.w0};
            row[1] = gw.a;
            row[2] = gw.b;
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
            u32x4* dst = (u32x4*)(a.obs + ((int64_t)step * B + g0) * 4 * 48);
            if (wave_games == kQuadGames) {
                const u32x4 p0 = stage[lane], p1 = stage[lane + 64], p2 = stage[lane + 128];
                st_nt(&dst[lane], p0, SECHS_NT_OBS);
                st_nt(&dst[lane + 64], p1, SECHS_NT_OBS);
                st_nt(&dst[lane + 128], p2, SECHS_NT_OBS);
            } else {
                const int pieces = wave_games * 12;  // lanes 0 .. 4 * wave_games - 1 are live
                for (int i = lane; i < pieces; i += 4 * wave_games) dst[i] = stage[i];
            }
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        }
        pp.mark(PH_OBS);
        const int64_t o = ((int64_t)step * B + g) * 4 + q;
        if (n == 0u) {  // a finished game stepped without auto-reset: nothing to play
            if (a.rewards) a.rewards[o] = 0;
            if (a.done && q == 0) a.done[(int64_t)step * B + g] = 1;
            continue;
        }
        // ---- DrunkHamster: legal[random_interval(n - 1)] for every seat
        const uint32_t idx = quad_draw(P, t, n - 1u, q);
        const uint32_t card = hand_get(h, idx);
        SN_DASSERT(idx < n && card < (uint32_t)C);  // the hand holds the card
        hand_del(h, idx);
        pp.mark(PH_DRAW);
        // ---- simultaneous placement, cards ascending (env.py:120-136)
        uint32_t k0 = (card << 8) | (heads_of(card) << 2) | (uint32_t)q;
        uint32_t k1 = qget<1>(k0), k2 = qget<2>(k0), k3 = qget<3>(k0);
        k0 = qget<0>(k0);
        qce(k0, k1), qce(k2, k3), qce(k0, k2), qce(k1, k3), qce(k1, k2);
        SN_DASSERT((k0 >> 8) < (k1 >> 8) && (k1 >> 8) < (k2 >> 8) && (k2 >> 8) < (k3 >> 8));  // four distinct cards
        uint32_t pen = 0u;
        {
            const uint32_t keys[4] = {k0, k1, k2, k3};
#pragma unroll
            for (int i = 0; i < 4; i++) {
                const uint32_t p = quad_place(rlo, rhi, keys[i] >> 8, (keys[i] >> 2) & 63u, q);
                pen += ((keys[i] & 3u) == (uint32_t)q) ? p : 0u;
            }
        }
        score += (int32_t)pen;
        n -= 1u;
        const bool done = n == 0u;  // env.py:246-249
        pp.mark(PH_RESOLVE);
        if (!(a.dbg & 2)) {
            const bool nt = SECHS_NT_MORE && !(a.dbg & 1);
            if (a.rewards) st_nt(&a.rewards[o], -(int32_t)pen, nt);
            if (a.actions_out) st_nt(&a.actions_out[o], (uint8_t)card, nt);
            if (a.done && q == 0) st_nt(&a.done[(int64_t)step * B + g], (uint8_t)(done ? 1 : 0), nt);
        }
        pp.mark(PH_STORE);
        if (done && auto_reset) {
            // GameSession.results.append(scores), then the next play_game(): _deal
            sres -= score;
            eps += 1;
            // np.random.shuffle(arange(C)): legacy Fisher-Yates from the end,
            // j = random_interval(i); one word per LDS round trip (the quad's
            // lanes do the same swap: same reads, same values written)
            for (int d = q; d < (C + 3) >> 2; d += 4) ((uint32_t*)deck)[d] = (uint32_t)d * 0x04040404u + 0x03020100u;
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
            uint32_t i = (uint32_t)C - 1u;
            while (i >= 1u) {  // quad-uniform
                const uint64_t w = P.peek8(t);
                uint32_t used = 0u;
#pragma unroll
                for (uint32_t kk = 0; kk < 8u; kk++) {
                    const bool act = i >= 1u;
                    const uint32_t m = 0xFFFFFFFFu >> __builtin_clz(i | 1u);
                    const uint32_t x = (uint32_t)(w >> (8u * kk)) & m;
                    const bool acc = act && x <= i;
                    const uint32_t j = acc ? x : i;
                    const uint8_t di = deck[i], dj = deck[j];
                    deck[i] = dj;
                    deck[j] = di;
                    i -= acc ? 1u : 0u;
                    used = act ? kk + 1u : used;
                }
                t += used;
            }
            pp.mark(PH_DEAL);
            // hand q = sorted(deck[10q : 10q + 10]), row q = [deck[C - 1 - q]] (env.py:106-110)
            {
                const uint16_t* hp = (const uint16_t*)(deck + 10 * q);
                uint32_t v[kHand];
#pragma unroll
                for (int k = 0; k < 5; k++) {
                    const uint32_t two = hp[k];
                    v[2 * k] = two & 0xFFu;
                    v[2 * k + 1] = two >> 8;
                }
                h = hand_from_cards(v);
                SN_DASSERT(hand_strict(h) && hand_len(h) == (uint32_t)kHand);  // ten distinct cards dealt
                const uint32_t rc = deck[C - 1 - q];
                rlo = rc;
                rhi = meta_row(rc);
                score = 0;
                n = kHand;
            }
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
            pp.mark(PH_HANDS);
        }
        if (fused) tw_finish();
    }
    if (fused) {  // the round in flight, then any rounds left over (more needy games than steps)
        tw_finish();
        while (tw_todo) {
            tw_issue();
            tw_finish();
        }
        if (q == 0 && twisted) {  // push the crossing (k_pipe_code's untwist levels, newest first)
            for (int k = kMt0Levels - 1; k > 0; k--) s.mt0[k * B + g] = s.mt0[(k - 1) * B + g];
            s.mt0[g] = my_old0;
        }
    }
    // ---- store the game back
    if (a.dbg & 4) return;  // timing diagnostics only
    s.hand[(int64_t)(q * 3 + 0) * B + g] = (uint32_t)h.lo;
    s.hand[(int64_t)(q * 3 + 1) * B + g] = (uint32_t)(h.lo >> 32);
    s.hand[(int64_t)(q * 3 + 2) * B + g] = h.hi;
    s.score[(int64_t)q * B + g] = score;
    s.row_lo[(int64_t)q * B + g] = rlo;
    s.row_hi[(int64_t)q * B + g] = rhi;
    if (auto_reset) s.sum_res[(int64_t)q * B + g] = sres;
    if (q == 0) {
        if (auto_reset) s.episodes[g] = eps;
        s.pabsc[(int64_t)a.pipe_cout * B + g] = P.c0 + t;  // read by k_mt_ahead on the other queue
        if (fused) {
            s.ptend[(int64_t)a.pipe_tout * B + g] = te0 + (twisted ? (uint32_t)kMtN : 0u);
            if (twisted) s.ptp[g] = kMtN;
        }
        if (bad_start || t > P.avail) atomicAdd(s.perr, 1u);  // a draw needed a word past the twisted end
    }
    pp.mark(PH_EPILOGUE);
    pp.flush(lane);
}

}  // namespace sechs

// sechs_state.h -- device-side game state shared by the env and MCS kernels.
//
// Device state is struct-of-arrays over games, so lane g of a wave reads
// element g of every array and each load/store instruction of a wave is one
// contiguous 256-B segment:
//   hand   [N][3][B] u32   sorted hand bytes: lo.lo32, lo.hi32, hi (sechs_device.h)
//   row_lo [4][B]    u32   cards 0..3 of each row
//   row_hi [4][B]    u32   card4 | len<<8 | heads<<16 | end<<24
//   score  [N][B]    i32   penalties this episode (env.py:32)
//   sum_res[N][B]    i32   sum of finished episodes' results (-penalty)
//   episodes [B]     i32
//   mt [B][624] u32 + mt_pos [B]   numpy-compat mode: per-game MT19937 (AoS,
//                                  so a lane's lazy twist walks its own lines)
//   ctr [B] u64                    philox mode: words consumed
#pragma once
#include <hip/hip_runtime.h>

#include <string>

#include "../../include/sechs.h"
#include "sechs_device.h"

namespace sechs {

// ============================================================================
// device state
// ============================================================================
struct DevState {
    int64_t B;
    int N, C, rng_mode, pad_;
    uint64_t seed, game_offset;
    uint32_t* hand;
    uint32_t* row_lo;
    uint32_t* row_hi;
    int32_t* score;
    int32_t* sum_res;
    int32_t* episodes;
    uint32_t* mt;
    uint32_t* mt_pos;
    uint64_t* ctr;
    uint32_t* mt0;   // [kMt0Levels][B] old-round mt[0] of the newest word-0 crossing (export of straddling
                     // codes), then the crossings before it (k_mt_ahead / k_pipe_code untwist, several rounds)
    u32x4* ring;     // [ring_w/16][B] low bytes of the words k_mt_prep twisted ahead
    int ring_w;      // ring words per game (multiple of 64), 0 = no ring
    int pad2_;
    // pipelined twist-ahead (k_mt_ahead / RingPipe, sechs_env.hip):
    u32x4* pring;    // [kPipeRing/64][B] 64-B chunks: byte of absolute stream word p at p mod kPipeRing (ring_byte)
    uint32_t* pabsc; // [kPipeSlots][B] consumer position after a play launch (by launch index mod kPipeSlots)
    uint32_t* ptend; // [kPipeSlots][B] end of the twisted words after a prep launch (the same)
    uint32_t* ptp;   // [B] twist pointer (MtGen's pos field), owned by k_mt_ahead
    uint32_t* perr;  // [1] play lanes that ran past the twisted words (must stay 0)
    u32x4* drec;     // [kDecRecords][kDecQuads][B] decode-ahead records (k_decode -> k_play<RNG_NUMPY_DEC>), one
                     // per episode: start position, per-step stream offsets, the draws, the dealt hands / rows
    // batched tournament (sn_league_config): per game the current game's
    // player count k and seat agents, k | agent(seat p) << (4 + 4p)
    uint32_t* lgs;   // [B]
    int lg_K, lg_lo, lg_hi, lg_pad;
    uint32_t* lmem;  // [4][B*N] card memory of MCSAgent seats (sn_league_step), word-major
    int32_t* lpc;    // [B*N] cards k_league_mcs chose for the step (in lmem's allocation)
    int32_t* lpf;    // [B] 1 (| 2: quirk Q6): lpc holds this step's non-external cards
};

constexpr int kMt0Levels = 8;    // word-0 crossings kept in mt0 (the decode-ahead span: up to seven rounds)
constexpr int kPipeSlots = 8;    // pabsc buffers (by play launch index mod 8; ptend uses 2, by twist parity)
constexpr int kDecSlot = kPipeSlots;  // pabsc slots kDecSlot + (G & 1): the decoder's position after decode G
constexpr int kDecRecords = 16;  // decode-ahead record ring (episodes; >= 2K + 2 for K <= 5)
constexpr int kDecQuads = 6;     // 16-B pieces per record (24 dwords, the layout at DecSrc)
constexpr int kTimingEvents = 6; // SN_OPT_TIMING events per launch: play, twist, decode (start, end)
constexpr int kPipeRing = 4096;  // ring bytes per game (>= the lead 600 K + a whole round's overshoot: 3 623 at K = 5)

// pring layout: 64-byte chunks interleaved over games -- stream positions
// 64 c .. 64 c + 63 of game g at chunk c * B + g -- so a twist wave's
// tempered bytes of 64 consecutive words fill one whole 64-B line (16-B
// chunks left 48 of every 64 bytes of each written line to other games:
// 4x the write traffic), and a play wave's 16-B window reads of 64
// consecutive games still cover one 4-KB run per instruction group.
// ring16: the u32x4 index of the 16-B unit u (positions 16 u .. 16 u + 15)
__host__ __device__ __forceinline__ int64_t ring16(uint32_t u, int64_t g, int64_t B) {
    u &= (uint32_t)(kPipeRing / 16 - 1);
    return ((int64_t)(u >> 2) * B + g) * 4 + (u & 3u);
}
// byte offset of stream position ri (mod kPipeRing) of game g
__host__ __device__ __forceinline__ int64_t ring_byte(uint32_t ri, int64_t g, int64_t B) {
    return ring16(ri >> 4, g, B) * 16 + (ri & 15u);
}constexpr int kPipeLead = 600;   // words k_mt_ahead keeps twisted ahead of the consumer (<= 624)
constexpr int kPipeWin = 240;    // of them, copied to LDS per lane at a k_play launch: a 4-player
                                  // episode draws 193.5 words, P(> 240) = 7e-6 per game (the rest come
                                  // from HBM); 304 -> 240 measured 7.46 -> 7.60 G env-steps/s interleaved

constexpr int kBlock = 256;
constexpr int kLeagueMaxPlayers = 6;  // tournament handles: 2..6 seats (agent ids packed 4 bits per seat)
constexpr int kLeagueMaxAgents = 16;
constexpr int kSplitMaxPlayers = 4;   // k_play_split: LDS for 4 staging + 4 producer waves
constexpr int kSplitEarly = 2;  // k_play_split: steps handed to the play waves before the rest is decoded
constexpr int kDeckStride = 108;  // 27 dwords: odd dword stride -> conflict-free LDS lanes
constexpr int kDealStride = 212;  // deck (108) + swap targets (104): 53 dwords, odd as well

// ---------------------------------------------------------------- rng glue
// PF = MT19937 refills prefetched ahead (MtGenT); Philox ignores it.
template <int MODE, int PF = 1>
struct RngOf;
template <int PF>
struct RngOf<RNG_NUMPY_MT, PF> {
    using T = MtGenT<PF>;
    static __device__ __forceinline__ void load(const DevState& s, int64_t g, T& r, ByteBuf& buf) {
        r.load(s.mt + g * kMtN, s.mt_pos[g], buf);
    }
    static __device__ __forceinline__ void store(const DevState& s, int64_t g, T& r, const ByteBuf& buf) {
        s.mt_pos[g] = r.save(buf);
    }
};
template <int PF>
struct RngOf<RNG_PHILOX, PF> {
    using T = PhiloxGen;
    static __device__ __forceinline__ void load(const DevState& s, int64_t g, T& r, ByteBuf& buf) {
        r.load((uint32_t)s.seed, (uint32_t)(s.seed >> 32), s.game_offset + (uint64_t)g, s.ctr[g], buf);
    }
    static __device__ __forceinline__ void store(const DevState& s, int64_t g, const T& r, const ByteBuf& buf) {
        s.ctr[g] = r.consumed(buf);
    }
};

// numpy-MT words for k_play from the ring k_mt_prep filled just before the
// launch: the low bytes of the next ring_w words of the game's stream, in
// 16-B chunks interleaved over games (chunk q of game g at ring[q*B + g], so
// a wave's lanes reading their q-th chunks read one contiguous 1-KB run).
// LDS = true: the lane copies its ring to its LDS slot at launch start (16
// coalesced loads per lane, one wait), so the step loop issues no global
// loads at all -- a global load there would wait behind every observation
// store still in flight (vmcnt counts loads and stores in issue order).
// LDS = false: chunks come from HBM, the next one prefetched.  A lane that
// runs the ring dry continues with MtGen from the in-place state (rare: the
// ring is sized for a launch's draws + ~6.5 sd).
// Past the ring (rare): the next 8 words of the stream from the in-place
// state -- `extra` twisted words first, then numpy's in-place twist of the
// next 8 (T stays 8-aligned; a crossed round saves the old mt[0]).  Out of
// line and by value, so the hot inlined paths carry none of it.
struct RingSlow {
    uint64_t bytes;
    uint32_t T, extra;
};

static __device__ __noinline__ RingSlow ring_slow8(uint32_t* st, uint32_t* mt0, uint32_t T, uint32_t extra) {
    RingSlow r;
    r.bytes = 0ull;
    if (extra) {  // replay: words [T - extra, T) mod 624
        const uint32_t from = (T >= extra) ? T - extra : T + kMtN - extra;
        const uint32_t k = min(8u, extra);
        for (uint32_t i = 0; i < k; i++) {
            const uint32_t idx = (from + i >= (uint32_t)kMtN) ? from + i - kMtN : from + i;
            r.bytes |= (uint64_t)(mt_temper(st[idx]) & 0xFFu) << (8u * i);
        }
        r.T = T, r.extra = extra - k;
        r.extra |= k << 16;  // count of bytes in r.bytes (< 8 only when replaying a short tail)
        return r;
    }
    const uint32_t i0 = (T == (uint32_t)kMtN) ? 0u : T;
    for (uint32_t i = 0; i < 8u; i++) {
        const uint32_t idx = i0 + i;
        const uint32_t a = st[idx];
        const uint32_t v = mt_mix(a, st[(idx + 1u == (uint32_t)kMtN) ? 0u : idx + 1u],
                                  st[(idx < (uint32_t)(kMtN - kMtM)) ? idx + kMtM : idx - (uint32_t)(kMtN - kMtM)]);
        if (idx == 0u) *mt0 = a;
        st[idx] = v;
        r.bytes |= (uint64_t)(mt_temper(v) & 0xFFu) << (8u * i);
    }
    r.T = i0 + 8u;
    r.extra = 8u << 16;
    return r;
}

// numpy-MT words for k_play from the ring k_mt_prep filled just before the
// launch: the low bytes of the next ring_w words of the game's stream, in
// 16-B chunks interleaved over games (chunk q of game g at ring[q*B + g], so
// a wave's lanes reading their q-th chunks read one contiguous 1-KB run).
// LDS = true: the lane copies its ring to its LDS slot at launch start (16
// coalesced loads per lane, one wait), so the step loop issues no global
// loads at all -- a global load there would wait behind every observation
// store still in flight (vmcnt counts loads and stores in issue order).
// LDS = false: chunks come from HBM, the next one prefetched.  A lane that
// runs the ring dry continues with ring_slow8 (rare: the ring is sized for a
// launch's draws + ~6.5 sd).
template <bool LDS>
struct RingGen {
    const u32x4* base;     // ring + g
    const uint8_t* lring;  // LDS copy (LDS = true)
    uint32_t* st;
    uint32_t* mt0;
    int64_t B;
    u32x4 c0, c1;          // chunks q, q + 1 (LDS = false)
    uint32_t q, nq, half;  // next chunk, chunks in the ring, next 8-B half of c0
    uint32_t rb;           // ring bytes not yet handed out
    uint32_t T, extra;     // twist position; twisted words past the ring

    __device__ __forceinline__ void load(const DevState& s, int64_t g, ByteBuf& buf, uint8_t* lds_slot) {
        const uint32_t code = s.mt_pos[g];
        T = code & 0x7FFu;
        const uint32_t rem = (code >> 16) & kMtCntMask;
        rb = (uint32_t)s.ring_w;  // k_mt_prep left rem >= ring_w
        extra = rem - rb;
        st = s.mt + g * kMtN;
        mt0 = s.mt0 + g;
        B = s.B;
        base = s.ring + g;
        nq = rb >> 4;
        q = 0u, half = 0u;
        if (LDS) {
            lring = lds_slot;
            for (uint32_t i = 0; i < nq; i++) {  // 8-B aligned slot: two ds_write_b64
                const u32x4 c = base[(int64_t)i * B];
                *(uint64_t*)(lds_slot + 16u * i) = (uint64_t)c.x | ((uint64_t)c.y << 32);
                *(uint64_t*)(lds_slot + 16u * i + 8u) = (uint64_t)c.z | ((uint64_t)c.w << 32);
            }
        } else {
            c0 = base[0];
            c1 = base[B];
        }
        buf.clear();
    }
    __device__ __forceinline__ uint32_t save(const ByteBuf& buf) { return T | ((rb + extra + buf.cnt) << 16); }
    __device__ __forceinline__ bool gen(ByteBuf& buf) {
        if (rb) {
            uint64_t v;
            if (LDS) {
                v = *(const uint64_t*)(lring + 8u * (2u * q + half));
                q += half;
            } else {
                v = half ? ((uint64_t)c0.z | ((uint64_t)c0.w << 32)) : ((uint64_t)c0.x | ((uint64_t)c0.y << 32));
                if (half) {
                    c0 = c1;
                    q += 1u;
                    c1 = base[(int64_t)min(q + 1u, nq - 1u) * B];
                }
            }
            buf.append(v, 8u);
            rb -= 8u;
            half ^= 1u;
            return true;
        }
        const RingSlow r = ring_slow8(st, mt0, T, extra);
        T = r.T;
        extra = r.extra & 0xFFFFu;
        buf.append(r.bytes, r.extra >> 16);
        return true;
    }
    __device__ __forceinline__ void topup(ByteBuf& buf) {
        if (buf.cnt <= 24u) gen(buf);
    }
    __device__ __forceinline__ void force(ByteBuf& buf) { gen(buf); }  // cnt == 0: always succeeds
};

// numpy-MT words for k_play from the pipelined ring: k_mt_ahead twisted the
// stream up to `tend` (593..600 words past the consumer position of the
// launch before) while the previous k_play ran.  The first kPipeWin of those
// bytes are copied to LDS at start (21 coalesced 1-KB loads per wave); reads
// are 8 bytes at any byte offset (two aligned ds_read_b64 + funnel shift).
// Past the window the bytes come from HBM.  A top-up (prefetch) never reads
// past `tend`; a draw that NEEDS a word past it would need one the next
// k_mt_ahead is twisting concurrently: it counts an error (perr, sticky,
// surfaced as SN_ERNG by sn_rollout) and draws zero bytes.  The host caps
// the launch length per player count (pipe_max_chunk, sechs_env.hip) so that
// two launches' draws exceed 592 words with probability < 1e-25 per game
// (exact tail of the geometric word counts).
struct PipeSlow {
    uint64_t bytes;
    uint32_t k;
};

static __device__ __noinline__ PipeSlow pipe_slow(const uint8_t* ring, int64_t B, int64_t g, uint32_t pos, uint32_t left,
                                                  uint32_t* err) {
    PipeSlow r;
    r.bytes = 0ull;
    r.k = min(8u, left);
    for (uint32_t i = 0; i < r.k; i++) {
        const uint32_t ri = (pos + i) & (uint32_t)(kPipeRing - 1);
        r.bytes |= (uint64_t)ring[ring_byte(ri, g, B)] << (8u * i);
    }
    if (r.k == 0u) {
        atomicAdd(err, 1u);
        r.k = 8u;
    }
    return r;
}

struct RingPipe {
    const uint8_t* slot;  // LDS window: chunk-aligned copy starting at the consumer's chunk
    const uint8_t* ring;
    uint32_t* err;
    int64_t B, g;
    uint32_t c0, off, take, win, avail;

    __device__ __forceinline__ void load(const DevState& s, int64_t gg, ByteBuf& buf, uint8_t* lds_slot, int cin, int tpar) {
        g = gg, B = s.B;
        c0 = s.pabsc[(int64_t)cin * B + g];
        // signed: a consumer past the twisted end (an earlier overrun) must
        // not read as a huge window of stale ring bytes
        const int32_t av = (int32_t)(s.ptend[(int64_t)tpar * B + g] - c0);
        if (av < 0) atomicAdd(s.perr, 1u);
        avail = (av < 0) ? 0u : (uint32_t)av;
        win = min(avail, (uint32_t)kPipeWin);
        off = c0 & 15u;
        slot = lds_slot;
        ring = (const uint8_t*)s.pring;
        err = s.perr;
        take = 0u;
        const uint32_t q0 = (c0 & (uint32_t)(kPipeRing - 1)) >> 4;
        const uint32_t nch = (off + win + 15u) >> 4;
        for (uint32_t i = 0; i < nch; i++) {
            const u32x4 c = s.pring[ring16(q0 + i, g, B)];
            *(uint64_t*)(lds_slot + 16u * i) = (uint64_t)c.x | ((uint64_t)c.y << 32);
            *(uint64_t*)(lds_slot + 16u * i + 8u) = (uint64_t)c.z | ((uint64_t)c.w << 32);
        }
        buf.clear();
    }
    // the same from an explicit position (k_decode: the decoder's own position, the twist's end)
    __device__ __forceinline__ void load_at(const DevState& s, int64_t gg, ByteBuf& buf, uint8_t* lds_slot, uint32_t c,
                                            uint32_t tend) {
        g = gg, B = s.B;
        c0 = c;
        const int32_t av = (int32_t)(tend - c0);
        if (av < 0) atomicAdd(s.perr, 1u);
        avail = (av < 0) ? 0u : (uint32_t)av;
        win = min(avail, (uint32_t)kPipeWin);
        off = c0 & 15u;
        slot = lds_slot;
        ring = (const uint8_t*)s.pring;
        err = s.perr;
        take = 0u;
        const uint32_t q0 = (c0 & (uint32_t)(kPipeRing - 1)) >> 4;
        const uint32_t nch = (off + win + 15u) >> 4;
        u32x4 v[(kPipeWin + 30) / 16];  // every load in flight before the first LDS write
#pragma unroll
        for (uint32_t i = 0; i < (uint32_t)((kPipeWin + 30) / 16); i++)
            if (i < nch) v[i] = s.pring[ring16(q0 + i, g, B)];
#pragma unroll
        for (uint32_t i = 0; i < (uint32_t)((kPipeWin + 30) / 16); i++)
            if (i < nch) {
                *(uint64_t*)(lds_slot + 16u * i) = (uint64_t)v[i].x | ((uint64_t)v[i].y << 32);
                *(uint64_t*)(lds_slot + 16u * i + 8u) = (uint64_t)v[i].z | ((uint64_t)v[i].w << 32);
            }
        buf.clear();
    }
    __device__ __forceinline__ uint32_t consumed(const ByteBuf& buf) const { return c0 + take - buf.cnt; }
    // forced = the buffer is empty and a draw needs a word now
    __device__ __forceinline__ bool gen(ByteBuf& buf, bool forced) {
        if (take + 8u <= win) {
            const uint32_t p = off + take, a8 = p & ~7u, sh = 8u * (p & 7u);
            const uint64_t lo = *(const uint64_t*)(slot + a8);
            const uint64_t hi = *(const uint64_t*)(slot + a8 + 8u);
            buf.append(sh ? ((lo >> sh) | (hi << (64u - sh))) : lo, 8u);
            take += 8u;
            return true;
        }
        const uint32_t left = (avail > take) ? avail - take : 0u;
        if (left == 0u && !forced) return false;  // prefetch stops at the twisted end
        const PipeSlow r = pipe_slow(ring, B, g, c0 + take, left, err);
        buf.append(r.bytes, r.k);
        take += r.k;
        return true;
    }
    __device__ __forceinline__ void topup(ByteBuf& buf) {
        if (buf.cnt <= 24u) gen(buf, false);
    }
    __device__ __forceinline__ void force(ByteBuf& buf) { gen(buf, true); }
};

// The pipelined ring read straight from HBM (k_decode, the decode-ahead
// producer): the next 8 bytes at any stream position from two 16-B units
// held in registers (the one holding the position and the next, loaded one
// unit ahead), the same words RingPipe hands out.  A top-up never reads past
// the twisted end; a draw that needs a word past it counts an overrun (perr,
// sticky) and takes zero bytes, as pipe_slow.
struct RingDirect {
    static constexpr int kAhead = 4;  // 16-B units in flight past the one being read (~64 words of draws)
    const u32x4* ring;
    uint32_t* err;
    int64_t B, g;
    uint32_t pos;  // stream position of the next byte not yet appended
    uint32_t end;  // twisted end (ptend)
    uint32_t unit;  // pos >> 4 (the unit `cur` holds)
    u32x4 cur, nx[kAhead];  // units unit, unit + 1 .. unit + kAhead (a register queue: static indices only)

    __device__ __forceinline__ void load(const DevState& s, int64_t gg, uint32_t c, uint32_t tend, ByteBuf& buf) {
        ring = s.pring, err = s.perr, B = s.B, g = gg;
        pos = c, end = tend, unit = c >> 4;
        cur = ring[ring16(unit, g, B)];
#pragma unroll
        for (int k = 0; k < kAhead; k++) nx[k] = ring[ring16(unit + 1u + (uint32_t)k, g, B)];
        buf.clear();
    }
    __device__ __forceinline__ uint32_t consumed(const ByteBuf& buf) const { return pos - buf.cnt; }
    __device__ __forceinline__ uint64_t peek8() const {
        const uint32_t off = pos & 15u, sh = 8u * (off & 7u);
        const uint64_t q0 = (uint64_t)cur.x | ((uint64_t)cur.y << 32), q1 = (uint64_t)cur.z | ((uint64_t)cur.w << 32);
        const uint64_t q2 = (uint64_t)nx[0].x | ((uint64_t)nx[0].y << 32);
        const uint64_t lo = (off >= 8u) ? q1 : q0, hi = (off >= 8u) ? q2 : q1;
        return sh ? ((lo >> sh) | (hi << (64u - sh))) : lo;
    }
    __device__ __forceinline__ void advance(uint32_t k) {
        pos += k;
        const uint32_t u = pos >> 4;  // (positions wrap at 2^32: a start-up consumer sits just below 0)
        if (u != unit) {              // at most one unit per call (k <= 8)
            unit = u;
            cur = nx[0];
#pragma unroll
            for (int q = 0; q + 1 < kAhead; q++) nx[q] = nx[q + 1];
            nx[kAhead - 1] = ring[ring16(unit + (uint32_t)kAhead, g, B)];
        }
    }
    // forced = the buffer is empty and a draw needs a word now
    __device__ __forceinline__ bool gen(ByteBuf& buf, bool forced) {
        const uint32_t left = ((int32_t)(end - pos) > 0) ? end - pos : 0u;
        if (left >= 8u) {
            buf.append(peek8(), 8u);
            advance(8u);
            return true;
        }
        if (left == 0u) {
            if (!forced) return false;  // prefetch stops at the twisted end
            atomicAdd(err, 1u);         // an overrun: the stream is lost, draw zeros
            buf.append(0ull, 8u);
            return true;
        }
        buf.append(peek8(), left);
        advance(left);
        return true;
    }
    __device__ __forceinline__ void topup(ByteBuf& buf) {
        if (buf.cnt <= 24u) gen(buf, false);
    }
    __device__ __forceinline__ void force(ByteBuf& buf) { gen(buf, true); }
};

// Phase (A) of deck_shuffle2 on the pipelined ring: the words are read
// straight from the LDS window by stream position (no byte buffer: appending
// and dropping a variable number of bytes is a long 64-bit shift chain), the
// next pass's 8 bytes prefetched while this pass decodes.  Same words, same
// targets as the generic form.
__device__ __forceinline__ uint64_t pipe_peek8(const RingPipe& r, uint32_t t) {
    const uint32_t p = r.off + t, a8 = p & ~7u, sh = 8u * (p & 7u);
    const uint64_t lo = *(const uint64_t*)(r.slot + a8);
    const uint64_t hi = *(const uint64_t*)(r.slot + a8 + 8u);
    return sh ? ((lo >> sh) | (hi << (64u - sh))) : lo;
}

// dummy: the byte a rejected word's store goes to (jslot[103] by default; k_decode, whose targets overlay
// the window's consumed head, passes a byte past the window's live bytes)
__device__ __forceinline__ void shuffle_targets(RingPipe& rng, ByteBuf& buf, uint8_t* jslot, int C,
                                                uint32_t dummy = 103u) {
    uint32_t t = rng.take - buf.cnt;  // next unconsumed byte (buffered bytes are re-read from the window)
    buf.clear();
    uint32_t i = (uint32_t)C - 1u;
    uint64_t w = 0ull;
    uint32_t valid = 8u;
    if (t + 8u <= rng.win) {
        w = pipe_peek8(rng, t);
    } else {
        const uint32_t left = (rng.avail > t) ? rng.avail - t : 0u;
        const PipeSlow r = pipe_slow(rng.ring, rng.B, rng.g, rng.c0 + t, left, rng.err);
        w = r.bytes, valid = r.k;
    }
    while (i >= 1u) {
        const uint32_t tn = t + 8u;
        const bool fast_next = tn + 8u <= rng.win;
        const uint64_t wn = fast_next ? pipe_peek8(rng, tn) : 0ull;  // speculative: a full pass
        uint32_t used = 0u, ii = i;
#pragma unroll
        for (uint32_t q = 0; q < 8u; q++) {
            const bool act = (q < valid) && (ii >= 1u);
            const uint32_t m = 0xFFFFFFFFu >> __builtin_clz(ii | 1u);
            const uint32_t x = (uint32_t)(w >> (8u * q)) & m;
            const bool acc = act && (x <= ii);
            jslot[acc ? (uint32_t)C - 1u - ii : dummy] = (uint8_t)x;
            ii -= acc ? 1u : 0u;
            used = act ? q + 1u : used;
        }
        i = ii;
        t += used;
        if (i >= 1u) {
            if (used == 8u && fast_next) {
                w = wn, valid = 8u;
            } else if (t + 8u <= rng.win) {
                w = pipe_peek8(rng, t), valid = 8u;
            } else {
                const uint32_t left = (rng.avail > t) ? rng.avail - t : 0u;
                const PipeSlow r = pipe_slow(rng.ring, rng.B, rng.g, rng.c0 + t, left, rng.err);
                w = r.bytes, valid = r.k;
            }
        }
    }
    rng.take = t;
}

// bytes of a lane's LDS window for RingPipe (chunk-aligned copy + 8 for the funnel's second read)
constexpr int kPipeSlot = ((kPipeWin + 15 + 15) / 16) * 16 + 8;

// bytes of a lane's LDS ring slot (+8: odd 8-B stride, conflict-free ds_read_b64 rows)
__host__ __device__ __forceinline__ int ring_lds_stride(int ring_w) { return ring_w + 8; }

template <int PF>
struct RngOf<RNG_NUMPY_RING, PF> {
    using T = RingGen<true>;
    static __device__ __forceinline__ void load(const DevState& s, int64_t g, T& r, ByteBuf& buf, uint8_t* slot) {
        r.load(s, g, buf, slot);
    }
    static __device__ __forceinline__ void store(const DevState& s, int64_t g, T& r, const ByteBuf& buf) {
        s.mt_pos[g] = r.save(buf);
    }
};
template <int PF>
struct RngOf<RNG_NUMPY_RING_HBM, PF> {
    using T = RingGen<false>;
    static __device__ __forceinline__ void load(const DevState& s, int64_t g, T& r, ByteBuf& buf, uint8_t*) {
        r.load(s, g, buf, nullptr);
    }
    static __device__ __forceinline__ void store(const DevState& s, int64_t g, T& r, const ByteBuf& buf) {
        s.mt_pos[g] = r.save(buf);
    }
};

// ---------------------------------------------------------------- tournament seat draw
// Tournament._choose_players (tournament.py:166-177) on the game's stream,
// right before its deal: num_players = np.random.choice(range(lo, hi+1)) =
// lo + random_interval(hi - lo) (no draw when lo == hi), then
// np.random.choice(K, num_players, replace=False) = permutation(K)[:k]
// (numpy legacy: shuffle(arange(K)), j = random_interval(i) for i = K-1..1).
// Returns k | agent(seat p) << (4 + 4p); K <= 16, k <= 6.
template <class R>
__device__ __forceinline__ uint32_t league_draw(R& rng, ByteBuf& buf, int K, int lo, int hi) {
    const uint32_t k = (uint32_t)lo + rng_interval(rng, buf, (uint32_t)(hi - lo));
    uint64_t perm = 0xFEDCBA9876543210ull;  // nibble i = i
    for (int i = K - 1; i >= 1; i--) {
        const uint32_t j = rng_interval(rng, buf, (uint32_t)i);
        const uint32_t si = 4u * (uint32_t)i, sj = 4u * j;
        const uint64_t a = (perm >> si) & 15ull, b = (perm >> sj) & 15ull;
        perm &= ~((15ull << si) | (15ull << sj));
        perm |= (b << si) | (a << sj);
    }
    return k | (uint32_t)((perm & ((1ull << (4u * k)) - 1ull)) << 4);
}

// ---------------------------------------------------------------- game in VGPRs
template <int N>
struct Game {
    Hand hand[N];
    Board b;
    int32_t score[N];
    uint32_t n;  // cards per hand (all seats hold the same count)
};

__device__ __forceinline__ Hand load_hand(const DevState& s, int p, int64_t g) {
    const int64_t B = s.B;
    Hand h;
    const uint32_t w0 = s.hand[(int64_t)(p * 3 + 0) * B + g];
    const uint32_t w1 = s.hand[(int64_t)(p * 3 + 1) * B + g];
    h.lo = (uint64_t)w0 | ((uint64_t)w1 << 32);
    h.hi = s.hand[(int64_t)(p * 3 + 2) * B + g];
    return h;
}

__device__ __forceinline__ Board load_board(const DevState& s, int64_t g) {
    const int64_t B = s.B;
    Board b;
    b.lo.x = s.row_lo[0 * B + g], b.lo.y = s.row_lo[1 * B + g], b.lo.z = s.row_lo[2 * B + g], b.lo.w = s.row_lo[3 * B + g];
    b.hi.x = s.row_hi[0 * B + g], b.hi.y = s.row_hi[1 * B + g], b.hi.z = s.row_hi[2 * B + g], b.hi.w = s.row_hi[3 * B + g];
    return b;
}

template <int N>
__device__ __forceinline__ void load_game(const DevState& s, int64_t g, Game<N>& G) {
#pragma unroll
    for (int p = 0; p < N; p++) {
        G.hand[p] = load_hand(s, p, g);
        G.score[p] = s.score[(int64_t)p * s.B + g];
    }
    G.b = load_board(s, g);
    G.n = hand_len(G.hand[0]);
}

template <int N>
__device__ __forceinline__ void store_game(const DevState& s, int64_t g, const Game<N>& G) {
    const int64_t B = s.B;
#pragma unroll
    for (int p = 0; p < N; p++) {
        s.hand[(int64_t)(p * 3 + 0) * B + g] = (uint32_t)G.hand[p].lo;
        s.hand[(int64_t)(p * 3 + 1) * B + g] = (uint32_t)(G.hand[p].lo >> 32);
        s.hand[(int64_t)(p * 3 + 2) * B + g] = G.hand[p].hi;
        s.score[(int64_t)p * B + g] = G.score[p];
    }
    s.row_lo[0 * B + g] = G.b.lo.x, s.row_lo[1 * B + g] = G.b.lo.y, s.row_lo[2 * B + g] = G.b.lo.z, s.row_lo[3 * B + g] = G.b.lo.w;
    s.row_hi[0 * B + g] = G.b.hi.x, s.row_hi[1 * B + g] = G.b.hi.y, s.row_hi[2 * B + g] = G.b.hi.z, s.row_hi[3 * B + g] = G.b.hi.w;
}

// 10-input sorting network: 29 compare-exchanges in 8 layers (Knuth, TAOCP
// 5.3.4; checked by the 0-1 principle over all 2^10 inputs).  Branch-free
// min/max in registers -- a wave sorts 64 hands in ~60 VALU.
__device__ __forceinline__ void sort10(uint32_t (&v)[10]) {
    constexpr int net[29][2] = {{0, 8}, {1, 9}, {2, 7}, {3, 5}, {4, 6}, {0, 2}, {1, 4}, {5, 8}, {7, 9}, {0, 3},
                                {2, 4}, {5, 7}, {6, 9}, {0, 1}, {3, 6}, {8, 9}, {1, 5}, {2, 3}, {4, 8}, {6, 7},
                                {1, 2}, {3, 5}, {4, 6}, {7, 8}, {2, 3}, {4, 5}, {6, 7}, {3, 4}, {5, 6}};
#pragma unroll
    for (int c = 0; c < 29; c++) {
        const uint32_t a = v[net[c][0]], b = v[net[c][1]];
        v[net[c][0]] = min(a, b);
        v[net[c][1]] = max(a, b);
    }
}

// sorted legal list from 10 distinct cards
__device__ __forceinline__ Hand hand_from_cards(uint32_t (&v)[10]) {
    sort10(v);
    Hand h;
    h.lo = (uint64_t)(v[0] | (v[1] << 8) | (v[2] << 16) | (v[3] << 24)) |
           ((uint64_t)(v[4] | (v[5] << 8) | (v[6] << 16) | (v[7] << 24)) << 32);
    h.hi = v[8] | (v[9] << 8) | 0xFFFF0000u;
    return h;
}

// env.py:99-112 _deal from a dealt deck: hand p = sorted(deck[10p:10p+10]),
// row r = [deck[C-1-r]]
template <int N, class D>
__device__ __forceinline__ void deal_from(const D& deck, int C, Game<N>& G) {
#pragma unroll
    for (int p = 0; p < N; p++) {
        uint32_t v[kHand];
#pragma unroll
        for (int k = 0; k < kHand; k++) v[k] = deck(kHand * p + k);
        G.hand[p] = hand_from_cards(v);
        G.score[p] = 0;
    }
    const uint32_t r0 = deck(C - 1), r1 = deck(C - 2), r2 = deck(C - 3), r3 = deck(C - 4);
    G.b.lo.x = r0, G.b.lo.y = r1, G.b.lo.z = r2, G.b.lo.w = r3;
    G.b.hi.x = meta_row(r0), G.b.hi.y = meta_row(r1), G.b.hi.z = meta_row(r2), G.b.hi.w = meta_row(r3);
    G.n = kHand;
}

// np.random.shuffle(arange(C)) (legacy Fisher-Yates from the end,
// j = random_interval(i)) in this lane's LDS slot, then deal.
//
// Word-synchronous form: instead of one rejection loop per draw, the lane
// walks its words in order, 8 per pass (the buffered ones first, then fresh
// refills), and every word advances the shuffle by at most one draw:
// accepted (x <= i) -> swap(i, x), i -= 1; rejected -> nothing.  That is
// exactly numpy's sequence of masked-rejection draws, and all lanes of a
// wave consume their words in lockstep (one refill per pass for every lane
// still shuffling).  A lane that finishes inside a pass keeps the unused
// words for its next draws.
//
// One LDS round trip per pass: the (up to) 8 swaps' positions are known
// before any deck value is (they depend on the words only), so the pass
// issues all 16 reads at once, forwards in registers the values the pass
// itself has already moved, and writes back in order.  A swap at step k
// writes positions i_k (never read again: later positions are all < i_k)
// and j_k; a later read aliases only an earlier j_k.
template <class R>
__device__ __forceinline__ uint32_t deck_shuffle(R& rng, ByteBuf& buf, uint8_t* deck, int C) {
    uint32_t passes = 0u;
    for (int i = 0; i < C; i += 4) *(uint32_t*)(deck + i) = (uint32_t)i * 0x01010101u + 0x03020100u;
    uint32_t i = (uint32_t)C - 1u;
    while (i >= 1u) {
        // a full 8-word window every pass (a pass over fewer words is a
        // wasted LDS round trip for the whole wave)
        if (__any(buf.cnt < 8u)) rng.topup(buf);
        if (buf.cnt == 0u) rng.force(buf);
        const uint32_t valid = min(buf.cnt, 8u);
        const uint64_t w = buf.b0;
        uint32_t I[8], J[8], Jm[8];
        uint32_t used = 0u, ii = i;
#pragma unroll
        for (uint32_t k = 0; k < 8u; k++) {
            const bool act = (k < valid) && (ii >= 1u);
            const uint32_t m = 0xFFFFFFFFu >> __builtin_clz(ii | 1u);
            const uint32_t x = (uint32_t)(w >> (8u * k)) & m;
            const bool acc = act && (x <= ii);
            I[k] = ii;
            J[k] = acc ? x : ii;      // rejected / past the end: a no-op self-swap
            Jm[k] = acc ? x : 0xFFu;  // positions this pass has written
            ii -= acc ? 1u : 0u;
            used = act ? k + 1u : used;
        }
        uint32_t DI[8], DJ[8];
#pragma unroll
        for (int k = 0; k < 8; k++) {
            DI[k] = deck[I[k]];
            DJ[k] = deck[J[k]];
        }
#pragma unroll
        for (int k = 1; k < 8; k++)
#pragma unroll
            for (int q = 0; q < k; q++) {  // ascending: the latest write wins
                DI[k] = (Jm[q] == I[k]) ? DI[q] : DI[k];
                DJ[k] = (Jm[q] == J[k]) ? DI[q] : DJ[k];
            }
#pragma unroll
        for (int k = 0; k < 8; k++) {
            deck[J[k]] = (uint8_t)DI[k];
            deck[I[k]] = (uint8_t)DJ[k];
        }
        i = ii;
        buf.drop(used);
        passes++;
    }
    return passes;
}

// Two-phase form of the same shuffle (deck_shuffle2, used by k_play and
// k_reset).  The swap targets depend on the words only, never on the deck,
// and the positions do not even depend on the words: step k swaps position
// i = C-1-k with j_k.  So
//  (A) shuffle_targets walks the words as above (8 per pass, full windows)
//      and only records j_k in the lane's target slot (one branch-free byte
//      store per word; a rejected word stores to a dummy byte);
//  (B) shuffle_apply then performs the swaps 8 steps per LDS round trip in
//      lockstep over the wave: the i side of a batch sits at the same
//      positions in every lane (conflict-free reads and writes), the values a
//      batch itself moves are forwarded in registers, and a batch is exactly
//      8 swaps (a pass of (A) averages ~5.6 accepted words).
// Same words consumed, same permutation: pinned by every deal parity test.
template <class R>
__device__ __forceinline__ void shuffle_targets(R& rng, ByteBuf& buf, uint8_t* jslot, int C) {
    uint32_t i = (uint32_t)C - 1u;
    while (i >= 1u) {
        if (__any(buf.cnt < 8u)) rng.topup(buf);
        if (buf.cnt == 0u) rng.force(buf);
        const uint32_t valid = min(buf.cnt, 8u);
        const uint64_t w = buf.b0;
        uint32_t used = 0u, ii = i;
#pragma unroll
        for (uint32_t q = 0; q < 8u; q++) {
            const bool act = (q < valid) && (ii >= 1u);
            const uint32_t m = 0xFFFFFFFFu >> __builtin_clz(ii | 1u);
            const uint32_t x = (uint32_t)(w >> (8u * q)) & m;
            const bool acc = act && (x <= ii);
            jslot[acc ? (uint32_t)C - 1u - ii : 103u] = (uint8_t)x;  // step C-1-i; 103 = dummy (C-2 <= 102)
            ii -= acc ? 1u : 0u;
            used = act ? q + 1u : used;
        }
        i = ii;
        buf.drop(used);
    }
}

__device__ __forceinline__ void shuffle_apply(uint8_t* deck, const uint8_t* jslot, int C) {
    // C % 8 == 0 (104 cards): every batch's i side is the 4-aligned run
    // [i0-7, i0] and its targets the 4-aligned run jslot[k0, k0+8), so they
    // move as dwords
    const bool al = (C & 7) == 0;
    for (int i0 = C - 1; i0 >= 1; i0 -= 8) {  // wave-uniform: steps i0, i0-1, .. (at most 8, all >= 1)
        const int ns = min(8, i0);
        const int k0 = C - 1 - i0;
        uint32_t I[8], J[8], DI[8], DJ[8];
        if (al) {
            const uint32_t j0 = *(const uint32_t*)(jslot + k0), j1 = *(const uint32_t*)(jslot + k0 + 4);
            const uint32_t d0 = *(const uint32_t*)(deck + i0 - 7), d1 = *(const uint32_t*)(deck + i0 - 3);
#pragma unroll
            for (int q = 0; q < 8; q++) {
                I[q] = (q < ns) ? (uint32_t)(i0 - q) : 0u;
                J[q] = (q < ns) ? (((q < 4 ? j0 : j1) >> (8 * (q & 3))) & 0xFFu) : 0u;
                // position i0 - q is byte 7 - q of the run: d1 holds bytes 4..7
                // (the padded last batch has i0 = 7: its pad position 0 is byte 0 of the run)
                DI[q] = ((q < 4 ? d1 : d0) >> (8 * (3 - (q & 3)))) & 0xFFu;
            }
#pragma unroll
            for (int q = 0; q < 8; q++) DJ[q] = deck[J[q]];
        } else {
#pragma unroll
            for (int q = 0; q < 8; q++) {
                // a batch past step i = 1 pads with self-swaps of position 0 (no-ops)
                I[q] = (q < ns) ? (uint32_t)(i0 - q) : 0u;
                J[q] = (q < ns) ? (uint32_t)jslot[k0 + q] : 0u;
            }
#pragma unroll
            for (int q = 0; q < 8; q++) {
                DI[q] = deck[I[q]];
                DJ[q] = deck[J[q]];
            }
        }
        // forwarding: within the batch only position j_m (m < q) was written
        // (with DI[m]); the i side is never read again (later j, i < i_m)
#pragma unroll
        for (int q = 1; q < 8; q++)
#pragma unroll
            for (int m = 0; m < q; m++) {  // ascending: the latest write wins
                DI[q] = (J[m] == I[q]) ? DI[m] : DI[q];
                DJ[q] = (J[m] == J[q]) ? DI[m] : DJ[q];
            }
#pragma unroll
        for (int q = 0; q < 8; q++) deck[J[q]] = (uint8_t)DI[q];
        if (al && ns == 8) {  // the final values of positions i0-7 .. i0
            *(uint32_t*)(deck + i0 - 3) = DJ[3] | (DJ[2] << 8) | (DJ[1] << 16) | (DJ[0] << 24);
            *(uint32_t*)(deck + i0 - 7) = DJ[7] | (DJ[6] << 8) | (DJ[5] << 16) | (DJ[4] << 24);
        } else {
#pragma unroll
            for (int q = 0; q < 8; q++) deck[I[q]] = (uint8_t)DJ[q];
        }
    }
}

// deck (kDeckStride bytes) followed by the swap-target slot
template <class R>
__device__ __forceinline__ void deck_shuffle2(R& rng, ByteBuf& buf, uint8_t* slot, int C) {
    shuffle_targets(rng, buf, slot + kDeckStride, C);
    for (int i = 0; i < C; i += 4) *(uint32_t*)(slot + i) = (uint32_t)i * 0x01010101u + 0x03020100u;
    shuffle_apply(slot, slot + kDeckStride, C);
}

// env.py:99-112 _deal from the shuffled deck in this lane's LDS slot
template <int N>
__device__ __forceinline__ void deal_from_deck(const uint8_t* deck, int C, Game<N>& G) {
    // hands from the first 10N bytes (4-B aligned slot), rows from the end
    constexpr int NW = (kHand * N + 3) / 4;
    uint32_t dw[NW];
#pragma unroll
    for (int q = 0; q < NW; q++) dw[q] = *(const uint32_t*)(deck + 4 * q);
#pragma unroll
    for (int p = 0; p < N; p++) {
        uint32_t v[kHand];
#pragma unroll
        for (int k = 0; k < kHand; k++) v[k] = (dw[(kHand * p + k) >> 2] >> (8 * ((kHand * p + k) & 3))) & 0xFFu;
        G.hand[p] = hand_from_cards(v);
        G.score[p] = 0;
    }
    const uint32_t r0 = deck[C - 1], r1 = deck[C - 2], r2 = deck[C - 3], r3 = deck[C - 4];
    G.b.lo.x = r0, G.b.lo.y = r1, G.b.lo.z = r2, G.b.lo.w = r3;
    G.b.hi.x = meta_row(r0), G.b.hi.y = meta_row(r1), G.b.hi.z = meta_row(r2), G.b.hi.w = meta_row(r3);
    G.n = kHand;
}

template <int N, class R>
__device__ __forceinline__ void deal_shuffle(R& rng, ByteBuf& buf, uint8_t* deck, int C, Game<N>& G) {
    deck_shuffle(rng, buf, deck, C);
    deal_from_deck<N>(deck, C, G);
}

// ---------------------------------------------------------------- observation
// env.py:188-212.  A seat's 48-byte row = [hand asc, -1 pad to 10][N]
// [lens][ends][heads][4x6 board, -1 pad][0 pad]; bytes 0..9 are the seat's
// hand bytes, bytes 10..47 are the same for every seat (game words).
struct GameWords {  // obs bytes 10..47 as words: w0 (bytes 12..15), a (16..31), b (32..47)
    uint32_t w0;
    u32x4 a, b;
};
template <bool SUMM>
__device__ __forceinline__ GameWords game_words(int N, const Board& b, uint32_t& w2hi) {
    // Built a row at a time as 6-byte groups (no per-byte selects): row r =
    // its packed cards 0..3 with the bytes past len forced to 0xFF (-1), card
    // 4 or 0xFF, then 0xFF; the four groups form the 24 board bytes X.
    const uint32_t lo[4] = {b.lo.x, b.lo.y, b.lo.z, b.lo.w};
    const uint32_t hi[4] = {b.hi.x, b.hi.y, b.hi.z, b.hi.w};
    uint64_t G[4];
#pragma unroll
    for (int r = 0; r < kRows; r++) {
        const uint32_t len = len_of(hi[r]);  // 1..5
        const uint32_t r4 = lo[r] | ((len >= 4u) ? 0u : (0xFFFFFFFFu << (8u * len)));
        const uint32_t b4 = (len == 5u) ? (hi[r] & 0xFFu) : 0xFFu;
        G[r] = (uint64_t)r4 | ((uint64_t)(b4 | 0xFF00u) << 32);
    }
    const uint64_t X0 = G[0] | (G[1] << 48), X1 = (G[1] >> 16) | (G[2] << 32), X2 = (G[2] >> 32) | (G[3] << 16);
    const uint64_t Y0 = (X0 >> 8) | (X1 << 56), Y1 = (X1 >> 8) | (X2 << 56), Y2 = X2 >> 8;  // X bytes 1..23 + 0
    const uint32_t nb = (uint32_t)N & 0xFFu;
    if (SUMM) {  // [10] N, [11..14] lens, [15..18] ends, [19..22] heads, [23..46] X, [47] 0
        const uint32_t L = ((hi[0] >> 8) & 0xFFu) | (hi[1] & 0xFF00u) | ((hi[2] << 8) & 0xFF0000u) | ((hi[3] << 16) & 0xFF000000u);
        const uint32_t H = ((hi[0] >> 16) & 0xFFu) | ((hi[1] >> 8) & 0xFF00u) | (hi[2] & 0xFF0000u) | ((hi[3] << 8) & 0xFF000000u);
        const uint32_t E = (hi[0] >> 24) | ((hi[1] >> 16) & 0xFF00u) | ((hi[2] >> 8) & 0xFF0000u) | (hi[3] & 0xFF000000u);
        w2hi = (nb << 16) | (L << 24);
        GameWords r;
        r.w0 = (L >> 8) | (E << 24);
        r.a = u32x4{(E >> 8) | (H << 24), (H >> 8) | ((uint32_t)X0 << 24), (uint32_t)Y0, (uint32_t)(Y0 >> 32)};
        r.b = u32x4{(uint32_t)Y1, (uint32_t)(Y1 >> 32), (uint32_t)Y2, (uint32_t)(Y2 >> 32)};
        return r;
    } else {  // [10] N, [11..34] X, zeros
        w2hi = (nb << 16) | ((uint32_t)X0 << 24);
        GameWords r;
        r.w0 = (uint32_t)Y0;
        r.a = u32x4{(uint32_t)(Y0 >> 32), (uint32_t)Y1, (uint32_t)(Y1 >> 32), (uint32_t)Y2};
        r.b = u32x4{(uint32_t)(Y2 >> 32), 0u, 0u, 0u};
        return r;
    }
}

// one seat's obs row of `stride` bytes (stride % 4 == 0, >= L)
__device__ __forceinline__ void store_obs_row(int8_t* dst, const Hand& h, uint32_t w2hi, const GameWords& gw,
                                              int stride) {
    const uint32_t w0 = (uint32_t)h.lo, w1 = (uint32_t)(h.lo >> 32), w2 = (h.hi & 0xFFFFu) | w2hi;
    if ((stride & 15) == 0 && (((uintptr_t)dst) & 15) == 0) {  // stride >= 48 here
        u32x4* d = (u32x4*)dst;
        d[0] = u32x4{w0, w1, w2, gw.w0};
        d[1] = gw.a;
        d[2] = gw.b;
        for (int i = 3; i < (stride >> 4); i++) d[i] = u32x4{0u, 0u, 0u, 0u};
    } else {
        uint32_t* d = (uint32_t*)dst;
        const int nw = stride >> 2;
        const uint32_t all[12] = {w0, w1, w2, gw.w0, gw.a.x, gw.a.y, gw.a.z, gw.a.w, gw.b.x, gw.b.y, gw.b.z, gw.b.w};
#pragma unroll
        for (int i = 0; i < 12; i++)
            if (i < nw) d[i] = all[i];
        for (int i = 12; i < nw; i++) d[i] = 0u;
    }
}


// ---------------------------------------------------------------- host helpers
sn_status set_error(sn_status st, const std::string& msg);
inline unsigned grid_for(int64_t n) { return (unsigned)((n + kBlock - 1) / kBlock); }

#define HIP_TRY(expr)                                                                                    \
    do {                                                                                                 \
        hipError_t e_ = (expr);                                                                          \
        if (e_ != hipSuccess) return ::sechs::set_error(SN_EHIP, std::string(#expr ": ") + hipGetErrorString(e_)); \
    } while (0)

// instantiate BODY with constexpr int NN = N_ for N in 1..10
// (SECHS_DEV_ONLY_N: a development build that instantiates one player count
// only, to iterate on kernels without the full 3-minute compile)
#ifdef SECHS_DEV_ONLY_N
#define SN_DISPATCH_N(N_, BODY)                                                              \
    if ((N_) == SECHS_DEV_ONLY_N) {                                                          \
        constexpr int NN = SECHS_DEV_ONLY_N;                                                 \
        BODY;                                                                                \
    } else                                                                                   \
        return ::sechs::set_error(SN_EUNSUPPORTED, "development build: one player count only");
#else
#define SN_DISPATCH_N(N_, BODY)                                                          \
    switch (N_) {                                                                        \
        case 1: { constexpr int NN = 1; BODY; } break;                                   \
        case 2: { constexpr int NN = 2; BODY; } break;                                   \
        case 3: { constexpr int NN = 3; BODY; } break;                                   \
        case 4: { constexpr int NN = 4; BODY; } break;                                   \
        case 5: { constexpr int NN = 5; BODY; } break;                                   \
        case 6: { constexpr int NN = 6; BODY; } break;                                   \
        case 7: { constexpr int NN = 7; BODY; } break;                                   \
        case 8: { constexpr int NN = 8; BODY; } break;                                   \
        case 9: { constexpr int NN = 9; BODY; } break;                                   \
        case 10: { constexpr int NN = 10; BODY; } break;                                 \
        default: return ::sechs::set_error(SN_EINVAL, "num_players out of range");      \
    }
#endif

}  // namespace sechs

struct sn_env {
    int device;
    int cus;          // compute units of `device` (persistent grids size by it)
    int chunk_steps;  // SN_OPT_CHUNK_STEPS
    int pipe;         // SN_OPT_PIPELINE
    int pipe_gpw;     // SN_OPT_PIPE_GPW: games per k_play wave on the pipelined path (32 or 64)
    int pipe_lead;    // SN_OPT_PIPE_LEAD: words k_mt_ahead keeps twisted ahead (kPipeLead; tests lower it)
    int lg_phase;     // tournament handle: env-steps since the games were dealt, mod 10 (-1: not dealt yet)
    int lg_kind[16];  // tournament handle: per agent SN_AGENT_* (sn_league_agents; all RANDOM by default)
    int lg_mpc[16], lg_mmax[16];  // MCSAgent agents: mc_per_card, mc_max
    int phase;        // every game's env-steps since its deal, mod 10, when they are in lockstep; -1 unknown
    int play_split;   // SN_OPT_PLAY_SPLIT: role-split k_play for lockstep DrunkHamster rollouts
    int twist_every;  // SN_OPT_TWIST_EVERY: a k_mt_ahead beside every K-th play launch (K = 1 .. 5)
    int tw_out;       // pipeline: ptend slot of the last twist
    uint64_t pphase;  // pipeline: play launches since it started
    int twist_round;  // SN_OPT_TWIST_ROUND: k_mt_ahead twists whole MT rounds (8 instead of 12 B of MT traffic per word)
    int pipe_serial;  // SECHS_PIPE_SERIAL=1 (diagnostics): each twist waits for the play launch before it (no overlap)
    int pl_cout;      // pabsc slot the last play launch wrote
    int pK;           // SN_OPT_TWIST_EVERY of the running pipeline
    hipEvent_t evt[2];  // after twist G, slot G mod 2
    int twist_skip;   // SN_OPT_TWIST_SKIP (tests only): steady twists after the first group twist nothing
    int pipe_dec;     // SN_OPT_PIPE_DEC: decode-ahead (k_decode + k_play<RNG_NUMPY_DEC>) where it applies
    int pdec;         // the running pipeline decodes ahead
    int64_t dec_e;    // decode-ahead: episodes the play launches finished since the pipeline start
    int64_t dec_next; // decode-ahead: the next episode k_decode will decode
    sechs::DevState s;
    // pipelined twist-ahead (sechs_env.hip launch_pipe): a k_mt_ahead for the
    // next play launch may be in flight on `side` (ev_prep) after a rollout
    int pvalid;         // ring + ptend/pabsc/ptp are the live RNG state (mt_pos is stale)
    uint64_t pcount;    // pipelined play launches so far
    hipStream_t side;
    hipStream_t side2;                      // decode-ahead: k_decode, concurrent with the twists on `side`
    hipEvent_t evd[2], ev_prep2;            // after decode G (slot G mod 2); behind side2 (sn_pipe_sync)
    hipEvent_t ev_prep, ev_main, ev_play;  // ev_play: after the last pipelined k_play (recorded on that call's stream)
    uint32_t* perr_host;                    // pinned, device-mapped mirror of s.perr (PlayArgs::perr_mirror)
    uint32_t* perr_host_dev;
    uint32_t* hbuf;      // one-game fast path (sn_step1 / sn_reset1): pinned, device-mapped exchange words
    uint32_t* hbuf_dev;
    // SN_OPT_TIMING: per-launch event pairs (k_play start/end on the launch
    // stream, k_mt_ahead and k_decode start/end on `side`), tcap launches, tn recorded
    hipEvent_t* tev;
    int* tev_tw;  // per recorded launch: bit 0 a twist ran beside it, bit 1 a decode after that (their events valid)
    int tcap, tn;
};

// Every entry point that reads or writes a handle's numpy-MT state other
// than the pipelined rollout itself calls this first (on its stream): waits
// for an in-flight k_mt_ahead and folds the pipeline back into mt_pos.
extern "C" sn_status sn_pipe_sync(sn_env* e, hipStream_t st);

// sechs_puct.hip -- "Alpha0.5" PUCT search (PUCTAgent / PolicyMCSAgent,
// agents/mcts.py:191-323) for many decisions at once on gfx950.
//
// The reference's rollouts of one decision form a dependent chain (each
// root choice reads the outcomes so far, mcts.py:276-302), so the batch
// runs over decisions: every launch advances rollout r of all D decisions
// by one step.  Per rollout step the host enqueues
//   k_puct_rows  -> candidate rows [D*N*n_cur][48], normalised exactly as
//                   SechsNimmtStateNormalization (utils/preprocessing.py:12-57)
//   policy MLP   -> logits (PyTorch-ROCm, bf16 or fp32: the north star's
//                   "policy/value net forward via PyTorch-ROCm")
//   k_puct_step  -> per seat: softmax; PUCT selection at the root (seat 0,
//                   first step: mcts.py:282-302) or a policy sample (:209-217);
//                   env step; at the last step the backup (mcts.py:100).
// Random words: Philox keyed (seed ^ step, game id / seat / rollout / phase).
// The root policy is evaluated once per decision (k_puct_root_rows): the
// reference re-evaluates it every rollout, with the same weights and the
// same input, so the probabilities are the same.
#include <hip/hip_bf16.h>

#include <algorithm>
#include <type_traits>

#include "sechs_state.h"

using namespace sechs;

constexpr int kRoWords = 48;     // rollout state words per decision
constexpr int kStatWords = 24;   // sums[10] counts[10] total min max
constexpr int kHistBins = 172;   // outcomes of seat 0: -171..0
constexpr int kRowLen = 48;      // 1 (action) + 47 (observation)

struct PuctArgs {
    int64_t D;                // decisions = B * popcount(seats_mask), or num_dec of a decision list
    uint32_t seats_mask, M;   // deciding seats, M = popcount
    const int32_t* dec;       // decision list (g * N + p per decision) or NULL (seats_mask)
    const uint32_t* lgs;      // tournament handle: per game k | agents..., the rollouts seat k players; NULL: N
    int N;                    // the handle's seats
    int n;                    // root hand size (all decisions in lockstep)
    int flags;                // 1: PUCT at the root (PUCTAgent), 0: sample it (PolicyMCSAgent)
    double c_puct;
    uint32_t seed_lo, seed_hi, step, rollout;
    const uint32_t* avail;    // [4][B*N] card memory (sn_mcs_memorize)
    int32_t* ro;              // [D][48] rollout games
    int32_t* stats;           // [D][24]
    int32_t* hist;            // [D][172]
    float* root_probs;        // [D][10]
    const uint32_t* step_dev; // decision counter in device memory (graph replays), else `step`
};

// the decision counter mixed into every Philox key of a decision: from
// device memory when the launches were captured into a graph (one capture
// replayed for every decision), else the launch argument
__device__ __forceinline__ uint32_t puct_step_of(const PuctArgs& a) { return a.step_dev ? *a.step_dev : a.step; }

__device__ __forceinline__ void dec_to_gp(const PuctArgs& a, int64_t d, int64_t& g, int& p) {
    if (a.dec) {  // a tournament agent's seats (sn_puct.dec_list)
        const int32_t gp = a.dec[d];
        g = gp / a.N;
        p = gp - (int)g * a.N;
        return;
    }
    g = d / a.M;
    uint32_t k = (uint32_t)(d - g * a.M), m = a.seats_mask;
    for (uint32_t i = 0; i < k; i++) m &= m - 1u;  // drop the k lowest deciding seats
    p = __builtin_ctz(m);
}

// players of game g: the agent's num_players = state[10] (mcts.py:62-64); a
// tournament game seats k <= N of the handle's N seats
__device__ __forceinline__ int players_of(const PuctArgs& a, int64_t g) { return a.lgs ? (int)(a.lgs[g] & 15u) : a.N; }

// utils/preprocessing.py:55-57 in float32, same operation order as torch
__device__ __forceinline__ float nrm(float x, float lo, float hi) {
    float t = x - lo;
    t = 2.0f * t;
    t = t / (hi - lo);
    return -1.0f + t;
}

template <typename T>
__device__ __forceinline__ T to_out(float v);
template <>
__device__ __forceinline__ float to_out<float>(float v) { return v; }
template <>
__device__ __forceinline__ __hip_bfloat16 to_out<__hip_bfloat16>(float v) { return __float2bfloat16(v); }

// one candidate row: [card, observation of a seat holding `h` on board `b`]
template <typename T>
__device__ __forceinline__ void write_row(T* dst, uint32_t card, const Hand& h, int N, const Board& b, int64_t st = 1) {
    dst[0] = to_out<T>(nrm((float)card, 0.f, 103.f));
#pragma unroll
    for (int k = 0; k < kHand; k++) {
        const uint32_t c = hand_get(h, (uint32_t)k);
        dst[(1 + k) * st] = to_out<T>(nrm(c == 0xFFu ? -1.f : (float)c, 0.f, 103.f));
    }
    dst[11 * st] = to_out<T>(nrm((float)N, 0.f, 6.f));
    const uint32_t lo[4] = {b.lo.x, b.lo.y, b.lo.z, b.lo.w};
    const uint32_t hi[4] = {b.hi.x, b.hi.y, b.hi.z, b.hi.w};
#pragma unroll
    for (int r = 0; r < kRows; r++) {
        dst[(12 + r) * st] = to_out<T>(nrm((float)len_of(hi[r]), 1.f, 5.f));
        dst[(16 + r) * st] = to_out<T>(nrm((float)end_of(hi[r]), 0.f, 103.f));
        dst[(20 + r) * st] = to_out<T>(nrm((float)heads_in(hi[r]), 1.f, 10.f));
#pragma unroll
        for (int i = 0; i < kThreshold; i++) {
            const float v = (i < 5 && (uint32_t)i < len_of(hi[r])) ? (float)card_at(lo[r], hi[r], i < 5 ? i : 0) : -1.f;
            dst[(24 + r * kThreshold + i) * st] = to_out<T>(nrm(v, 0.f, 103.f));
        }
    }
}

__device__ __forceinline__ Hand ro_hand(const int32_t* ro, int q) {
    Hand h;
    h.lo = (uint32_t)ro[8 + 3 * q] | ((uint64_t)(uint32_t)ro[9 + 3 * q] << 32);
    h.hi = (uint32_t)ro[10 + 3 * q];
    return h;
}
__device__ __forceinline__ Board ro_board(const int32_t* ro) {
    Board b;
    b.lo = u32x4{(uint32_t)ro[0], (uint32_t)ro[1], (uint32_t)ro[2], (uint32_t)ro[3]};
    b.hi = u32x4{(uint32_t)ro[4], (uint32_t)ro[5], (uint32_t)ro[6], (uint32_t)ro[7]};
    return b;
}

// ---------------------------------------------------------------- root
template <typename T>
__global__ void k_puct_root_rows(DevState s, PuctArgs a, T* rows) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= a.D * a.n) return;
    const int64_t d = i / a.n;
    const uint32_t k = (uint32_t)(i - d * a.n);
    int64_t g;
    int p;
    dec_to_gp(a, d, g, p);
    const Hand h = load_hand(s, p, g);
    write_row<T>(rows + i * kRowLen, hand_get(h, k), h, players_of(a, g), load_board(s, g));
}

// softmax(dim=0) of the root logits (mcts.py:227) and empty statistics
__global__ void k_puct_init(PuctArgs a, const float* logits) {
    const int64_t d = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (d >= a.D) return;
    const float* x = logits + d * a.n;
    float m = x[0];
    for (int k = 1; k < a.n; k++) m = fmaxf(m, x[k]);
    float e[kHand], sum = 0.f;
#pragma unroll
    for (int k = 0; k < kHand; k++) {
        e[k] = (k < a.n) ? __expf(x[k < a.n ? k : 0] - m) : 0.f;
        sum += e[k];
    }
#pragma unroll
    for (int k = 0; k < kHand; k++) a.root_probs[d * kHand + k] = (k < a.n) ? e[k] / sum : 0.f;
    for (int w = 0; w < kStatWords; w++) a.stats[d * kStatWords + w] = 0;
    a.stats[d * kStatWords + 21] = 1;     // min (set by the first backup)
    a.stats[d * kStatWords + 22] = -1000;  // max
    for (int b = 0; b < kHistBins; b++) a.hist[d * kHistBins + b] = 0;
}

// ---------------------------------------------------------------- rollouts
// _draw_env + _deal_hands (mcts.py:108-127): the decider is seat 0 of the
// rollout game, opponents are dealt from its memory
template <int N>
__device__ __forceinline__ void deal_one(const DevState& s, const PuctArgs& a, int64_t d, uint32_t rollout, int32_t* ro) {
    int64_t g;
    int p;
    dec_to_gp(a, d, g, p);
    const int64_t DN = s.B * N, dn = g * N + p;
    u32x4 av = {a.avail[dn], a.avail[DN + dn], a.avail[2 * DN + dn], a.avail[3 * DN + dn]};
    const uint64_t gid = s.game_offset + (uint64_t)g;
    PhiloxGen gen;
    ByteBuf buf;
    gen.load(a.seed_lo ^ puct_step_of(a), a.seed_hi, ((uint64_t)(uint32_t)gid << 32) | ((uint64_t)p << 28) | ((uint64_t)rollout << 8),
             0ull, buf);
    const Board b = load_board(s, g);
    const Hand me = load_hand(s, p, g);
    const uint32_t n = (uint32_t)a.n;
    ro[0] = b.lo.x, ro[1] = b.lo.y, ro[2] = b.lo.z, ro[3] = b.lo.w;
    ro[4] = b.hi.x, ro[5] = b.hi.y, ro[6] = b.hi.z, ro[7] = b.hi.w;
    ro[8] = (int32_t)(uint32_t)me.lo, ro[9] = (int32_t)(uint32_t)(me.lo >> 32), ro[10] = (int32_t)me.hi;
    uint32_t left = set_count(av);
    const int kp = players_of(a, g);
#pragma unroll
    for (int q = 1; q < N; q++) {
        u32x4 set = {0u, 0u, 0u, 0u};
        for (uint32_t i = 0; i < n && left > 0u && q < kp; i++) {
            const uint32_t k = rng_interval(gen, buf, left - 1u);
            const uint32_t c = set_select(av, k);
            av = clear_bit(av, c);
            set = set_bit(set, c);
            left--;
        }
        const Hand h = hand_from_set(set);  // seats past k: empty (0xFF), they play nothing
        ro[8 + 3 * q] = (int32_t)(uint32_t)h.lo, ro[9 + 3 * q] = (int32_t)(uint32_t)(h.lo >> 32), ro[10 + 3 * q] = (int32_t)h.hi;
    }
    ro[40] = 0;   // outcome
    ro[41] = -1;  // first move (index into the root's legal list)
}

template <int N>
__global__ void k_puct_deal(DevState s, PuctArgs a) {
    const int64_t d = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (d >= a.D) return;
    deal_one<N>(s, a, d, a.rollout, a.ro + d * kRoWords);
}

// rollouts r0 .. r0 + nr - 1 of every decision in one launch (nr x D lanes
// instead of D: the deal is a latency-bound chain of Philox draws per lane),
// rollout r's state at ro_out + ((r - r0) D + d) kRoWords -- the rollout then
// runs on that slice in place (sn_puct.rollouts pointed at it)
template <int N>
__global__ void k_puct_deal_batch(DevState s, PuctArgs a, uint32_t r0, int nr, int32_t* ro_out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= a.D * nr) return;
    const int64_t k = i / a.D, d = i - k * a.D;
    deal_one<N>(s, a, d, r0 + (uint32_t)k, ro_out + i * kRoWords);
}

// candidate rows of every seat of every rollout game: row (d, q, k)
template <typename T>
__global__ void k_puct_rows(PuctArgs a, int N, int n_cur, T* rows) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t per_d = (int64_t)N * n_cur;
    if (i >= a.D * per_d) return;
    const int64_t d = i / per_d;
    const int rem = (int)(i - d * per_d);
    const int q = rem / n_cur, k = rem - q * n_cur;
    const int32_t* ro = a.ro + d * kRoWords;
    int kp = N;
    if (a.lgs) {
        int64_t g;
        int p;
        dec_to_gp(a, d, g, p);
        kp = players_of(a, g);
    }
    if (q >= kp) {  // an absent seat of a smaller tournament game: a dummy row (its logits are never read)
#pragma unroll
        for (int j = 0; j < kRowLen; j++) rows[i * kRowLen + j] = to_out<T>(0.f);
        return;
    }
    const Hand h = ro_hand(ro, q);
    write_row<T>(rows + i * kRowLen, hand_get(h, (uint32_t)k), h, kp, ro_board(ro));
}

// ---------------------------------------------------------------- fused rollout MLP
// The rollout policy net MultiHeadedMLP(48, (H, H2), (1,)) (utils/nets.py:100-132)
// per candidate row r = [card, obs of its seat]:
//   h1  = relu(W1 [card, obs] + b1)                 (layer 1)
//   h2  = relu(W2 h1 + b2)                          (layer 2)
//   out = wh . h2 + bh                              (head: the policy logit)
// The obs part of layer 1 is shared by a seat's candidates: base[seat] =
// W1[:, 1:] obs + b1 once per seat (phase 2 of k_puct_mlp_seats, MFMA), and
// mlp_tile does the rest for a tile of 64 rows per wave in registers:
// h1[k][r] = relu(base[seat(r)][k] + card(r) * w1c[k]) built straight into
// the B fragments of v_mfma_f32_32x32x16_bf16 (bf16, the rounding of the
// reference-shaped PyTorch split path), layer 2 as 4 x 7 MFMA tiles per 32
// rows against W2 staged in LDS (bias b2 = the column against the ones
// feature h1[H] = 1), ReLU + bf16 rounding (the layer's output dtype in the
// PyTorch path), then the head as a dot with wh over each lane's 16
// accumulator rows and one cross-half lane swap.  The [features][rows]
// activations of both layers never reach HBM: per row 4 B of card in, 4 B of
// f32 logit out, plus the seat's base row (224 B, shared by its n_cur rows).
// Shapes: K = 112 (7 k-steps of 16: H <= 111 features + the ones feature),
// M = 128 (4 tiles of 32: H2 <= 127 outputs + the ones pass-through row).
constexpr int kMlpK = 112;           // layer-2 inputs (padded)
constexpr int kMlpM = 128;           // layer-2 outputs (padded)
constexpr int kMlpLdsK = kMlpK + 8;  // LDS row stride of W2 (240 B: 60 dwords, lanes o spread over the banks)

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_t;
typedef __attribute__((ext_vector_type(16))) float f32x16_t;

typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2_t;
typedef __attribute__((ext_vector_type(2))) float f32x2_t;

// single-instruction ReLU and f32 FMA: plain fmaxf on an MFMA result gets a
// canonicalising v_max in front, and adjacent fmaf calls get SLP-packed into
// v_pk_fma_f32, which costs more than two v_fma_f32 beside MFMAs
// (MI355X_MICROARCH.md, issue-cost rows)
__device__ __forceinline__ float relu_f32(float v) {
    float r;
    asm("v_max_f32 %0, 0, %1" : "=v"(r) : "v"(v));
    return r;
}
// ReLU of a bf16 pair after rounding (the same as rounding after the ReLU:
// rounding keeps the sign): a signed 16-bit max with 0 per half, one
// v_pk_max_i16 for two values (-0.0 = 0x8000 becomes +0)
__device__ __forceinline__ uint32_t relu_bf16x2(uint32_t p) {
    uint32_t r;
    asm("v_pk_max_i16 %0, %1, 0" : "=v"(r) : "v"(p));
    return r;
}
__device__ __forceinline__ float fma_f32(float a, float b, float c) {
    float r;
    asm("v_fma_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}

// two f32 -> one bf16 pair, round to nearest even (v_cvt_pk_bf16_f32)
__device__ __forceinline__ uint32_t pack_bf16(float lo, float hi) {
    const bf16x2_t v = {(__bf16)lo, (__bf16)hi};
    return __builtin_bit_cast(uint32_t, v);
}

// One 64-row tile of the rollout MLP for a wave: rows col (nt = 0) and
// 32 + col (nt = 1) of the tile, their layer-1 base rows (bf16 [112]) and
// card features x.  Layer 1's card column + ReLU builds the MFMA B fragments
// (f32 fma, bf16 rounding as the GEMM's output), layer 2 runs as 4 x 7
// v_mfma_f32_32x32x16_bf16 against W2 in LDS, its ReLU'd bf16 outputs are
// dotted with the head (bf16 pairs, v_dot2 in f32) and the two halves of
// the wave summed.  sH2: the head as bf16 pairs, o = 2i, 2i + 1.
template <int NT>
__device__ __forceinline__ void mlp_tile(const uint16_t* const (&brow)[NT], const float (&x)[NT], const uint16_t* sW,
                                         const float* sC, const uint32_t* sH2, int col, int half, float (&out)[NT]) {
    f32x16_t acc[4][NT];
    // one k-step: the B fragments (16 features of the two 32-row halves), then 4 x 2 MFMAs
    auto kstep = [&](int ks, bool first) {
        const int k0 = 16 * ks + 8 * half;  // this lane's 8 features of the k-step
        // the k-step's four W2 A fragments issued first, their LDS latency under the B fragments'
        // VALU (the scheduler would otherwise sink each load to just before its MFMA pair)
        bf16x8_t af[4];
#pragma unroll
        for (int mt = 0; mt < 4; mt++)
            af[mt] = __builtin_bit_cast(bf16x8_t, *(const uint4*)&sW[(32 * mt + col) * kMlpLdsK + k0]);
        __builtin_amdgcn_sched_barrier(0);
        const float4 wa = *(const float4*)&sC[k0], wb = *(const float4*)&sC[k0 + 4];
        const float w[8] = {wa.x, wa.y, wa.z, wa.w, wb.x, wb.y, wb.z, wb.w};
        bf16x8_t bfr[NT];
#pragma unroll
        for (int nt = 0; nt < NT; nt++) {
            const uint4 bv = *(const uint4*)(brow[nt] + k0);
            const uint32_t bw[4] = {bv.x, bv.y, bv.z, bv.w};
            uint32_t hb[4];
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const float lo = fma_f32(x[nt], w[2 * j], __uint_as_float(bw[j] << 16));
                const float hi = fma_f32(x[nt], w[2 * j + 1], __uint_as_float(bw[j] & 0xFFFF0000u));
                hb[j] = relu_bf16x2(pack_bf16(lo, hi));
            }
            bfr[nt] = __builtin_bit_cast(bf16x8_t, make_uint4(hb[0], hb[1], hb[2], hb[3]));
        }
#pragma unroll
        for (int mt = 0; mt < 4; mt++) {
            const f32x16_t zero = {};
#pragma unroll
            for (int nt = 0; nt < NT; nt++)
                acc[mt][nt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[mt], bfr[nt], first ? zero : acc[mt][nt], 0, 0, 0);
        }
    };
    kstep(0, true);  // the accumulators start from the first k-step's products (no zeroing pass)
#pragma unroll 1
    for (int ks = 1; ks < kMlpK / 16; ks++) kstep(ks, false);
    // epilogue: ReLU, bf16 rounding, head dot over this lane's outputs o
    // (C layout: o = 32 mt + 8 g + 4 half + i, i = 0..3), then the other half's
    // (the head pairs of an output tile read once for both row halves, the four issued together;
    // each half's sum in the same mt, g order as before)
    float sum[NT];
#pragma unroll
    for (int nt = 0; nt < NT; nt++) sum[nt] = 0.f;
#pragma unroll
    for (int mt = 0; mt < 4; mt++) {
        uint2 hw[4];
#pragma unroll
        for (int g = 0; g < 4; g++) hw[g] = *(const uint2*)&sH2[(32 * mt + 8 * g + 4 * half) / 2];
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int g = 0; g < 4; g++)
#pragma unroll
            for (int nt = 0; nt < NT; nt++) {
                const uint32_t p0 = relu_bf16x2(pack_bf16(acc[mt][nt][4 * g], acc[mt][nt][4 * g + 1]));
                const uint32_t p1 = relu_bf16x2(pack_bf16(acc[mt][nt][4 * g + 2], acc[mt][nt][4 * g + 3]));
                sum[nt] = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2_t, p0),
                                                          __builtin_bit_cast(bf16x2_t, hw[g].x), sum[nt], false);
                sum[nt] = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2_t, p1),
                                                          __builtin_bit_cast(bf16x2_t, hw[g].y), sum[nt], false);
            }
    }
#pragma unroll
    for (int nt = 0; nt < NT; nt++) out[nt] = sum[nt] + __shfl_xor(sum[nt], 32);
}

// the head as bf16 pairs in LDS (its values are bf16 weights: exact)
__device__ __forceinline__ void load_head_pairs(const float* head, uint32_t* sH2) {
    for (int i = threadIdx.x; i < kMlpM / 2; i += blockDim.x) sH2[i] = pack_bf16(head[2 * i], head[2 * i + 1]);
}

// np.median of all outcomes so far, from the histogram (kth smallest): one
// pass over the 172 bins as 43 16-B loads (issued ahead of the scan, no
// data-dependent exit: the scan's result is fixed once both ranks are found)
__device__ double hist_median(const int32_t* hist, int32_t total) {
    static_assert(kHistBins % 4 == 0, "16-B histogram rows");
    const int32_t k0 = (total - 1) / 2, k1 = total / 2;
    int32_t acc = 0, v0 = 0, v1 = 0;
    bool got0 = false, got1 = false;
    const int4* h4 = reinterpret_cast<const int4*>(hist);
#pragma unroll 11
    for (int c = 0; c < kHistBins / 4; c++) {
        const int4 w = h4[c];
        const int32_t cs[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const int32_t b = 4 * c + j - 171;
            const bool h0 = !got0 && acc + cs[j] > k0, h1 = !got1 && acc + cs[j] > k1;
            v0 = h0 ? b : v0, got0 = got0 || h0;
            v1 = h1 ? b : v1, got1 = got1 || h1;
            acc += cs[j];
        }
    }
    return 0.5 * ((double)v0 + (double)v1);
}

// hist_median over the L lanes of a decision (step_seat's lanes lead .. lead + L - 1,
// every one calling it): lane q scans bins [kChunk q, kChunk (q + 1)) -- its count,
// an exclusive prefix over the lanes by shuffles, then the lane holding rank k0
// (k1) finds its bin -- a quarter (L = 4) of the serial scan's loads and VALU on
// every lane.  Same value as hist_median.
template <int L>
__device__ __forceinline__ double hist_median_lanes(const int32_t* hist, int32_t total, int q, int lead) {
    constexpr int kChunk = ((kHistBins + 4 * L - 1) / (4 * L)) * 4;  // bins per lane, 4-aligned (L = 4: 44)
    const int32_t k0 = (total - 1) / 2, k1 = total / 2;
    int32_t mine = 0;
    const int4* h4 = reinterpret_cast<const int4*>(hist + kChunk * q);
#pragma unroll 2
    for (int c = 0; c < kChunk / 4; c++) {  // kHistBins % 4 == 0: whole int4 pieces
        const int4 w = (kChunk * q + 4 * c < kHistBins) ? h4[c] : make_int4(0, 0, 0, 0);
        mine += w.x + w.y + w.z + w.w;
    }
    int32_t pre = 0;  // outcomes in the lanes before this one
#pragma unroll
    for (int r = 0; r < L - 1; r++) {
        const int32_t c = __shfl(mine, lead + r);
        pre += (r < q) ? c : 0;
    }
    int32_t acc = pre, v0 = INT32_MIN, v1 = INT32_MIN;
    if (pre <= k1 && pre + mine > k0) {  // this lane holds rank k0 or k1: its bins again (L1)
#pragma unroll 2
        for (int c = 0; c < kChunk / 4; c++) {
            const int4 w = (kChunk * q + 4 * c < kHistBins) ? h4[c] : make_int4(0, 0, 0, 0);
            const int32_t cs[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const int32_t b = kChunk * q + 4 * c + j - 171;
                if (acc <= k0 && acc + cs[j] > k0) v0 = b;
                if (acc <= k1 && acc + cs[j] > k1) v1 = b;
                acc += cs[j];
            }
        }
    }
#pragma unroll
    for (int r = 0; r < L; r++) {  // the owners' bins to every lane of the decision
        v0 = max(v0, __shfl(v0, lead + r));
        v1 = max(v1, __shfl(v1, lead + r));
    }
    return 0.5 * ((double)v0 + (double)v1);
}

// PUCTAgent._compute_pucts + argmax (mcts.py:282-315) with numpy's float
// types: c_puct * probs is float32 (a Python float times a float32 array);
// (n_total + 1e-9) ** 0.5 is a numpy float64 scalar, which promotes the
// product to float64 (numpy >= 2 promotion, the version the golden vectors
// were recorded with); q and the division by (1 + n) are float64
// med_all: np.median of all outcomes (read only when st[20] >= 10)
__device__ __forceinline__ int puct_choose_med(const int32_t* st, double med_all, const float* probs, int n,
                                               double c_puct, double* pucts_out) {
    const int32_t total = st[20];
    int32_t n_total = 0;
    for (int k = 0; k < n; k++) n_total += st[10 + k];
    double mx, mn, med;
    if (total < 10) {
        mx = 0.0, mn = -10.0, med = -5.0;  // _normalize_q fallback (quirk Q8)
    } else {
        mx = (double)st[22], mn = (double)st[21], med = med_all;
    }
    const double sq = sqrt((double)n_total + 1e-9);
    double best = -__builtin_inf();
    int choice = 0;
    for (int k = 0; k < n; k++) {
        const int32_t cnt = st[10 + k];
        double q = cnt ? (double)st[k] / (double)cnt : med;
        q = (q - mn) / (mx - mn);         // max == min: NaN for every move (quirk Q7)
        q = (q < 0.0) ? 0.0 : (q > 1.0) ? 1.0 : q;  // np.clip keeps NaN
        const double t = (double)((float)c_puct * probs[k]) * sq;
        const double v = q + t / (1.0 + (double)cnt);
        if (pucts_out) pucts_out[k] = v;
        if (v > best) best = v, choice = k;  // strict '>': NaN never wins, index 0 stays
    }
    return choice;
}

// puct_choose_med over the L lanes of a decision (lane q scores moves k = q, q + L, ..;
// every lane of the decision calls it, lead = its first lane): the same f64 arithmetic
// per move, the counts' sum and the first strict maximum (ties to the lower index, NaN
// never wins, move 0 when nothing does) combined by shuffles.  Same choice.
template <int L>
__device__ __forceinline__ int puct_choose_lanes(const int32_t* st, double med_all, const float* probs, int n,
                                                 double c_puct, int q, int lead) {
    constexpr int KL = (kHand + L - 1) / L;
    int32_t cnt[KL], sum[KL];
    float pr[KL];
    int32_t n_total = 0;
#pragma unroll
    for (int j = 0; j < KL; j++) {
        const int k = q + L * j;
        const bool on = k < n;
        cnt[j] = on ? st[10 + k] : 0;
        sum[j] = on ? st[k] : 0;
        pr[j] = on ? probs[k] : 0.f;
        n_total += cnt[j];
    }
#pragma unroll
    for (int r = 1; r < L; r <<= 1) n_total += __shfl_xor(n_total, r);  // lanes lead .. lead + L - 1 (aligned)
    const int32_t total = st[20];
    double mx, mn, med;
    if (total < 10) {
        mx = 0.0, mn = -10.0, med = -5.0;  // _normalize_q fallback (quirk Q8)
    } else {
        mx = (double)st[22], mn = (double)st[21], med = med_all;
    }
    const double sq = sqrt((double)n_total + 1e-9);
    double best = -__builtin_inf();
    int choice = 0;
#pragma unroll
    for (int j = 0; j < KL; j++) {
        const int k = q + L * j;
        if (k < n) {
            double qv = cnt[j] ? (double)sum[j] / (double)cnt[j] : med;
            qv = (qv - mn) / (mx - mn);
            qv = (qv < 0.0) ? 0.0 : (qv > 1.0) ? 1.0 : qv;
            const double t = (double)((float)c_puct * pr[j]) * sq;
            const double v = qv + t / (1.0 + (double)cnt[j]);
            if (v > best) best = v, choice = k;
        }
    }
#pragma unroll
    for (int r = 1; r < L; r <<= 1) {
        const double ob = __shfl_xor(best, r);
        const int oc = __shfl_xor(choice, r);
        const bool take = ob > best || (ob == best && oc < choice);
        best = take ? ob : best;
        choice = take ? oc : choice;
    }
    (void)lead;
    return choice;
}

__device__ int puct_choose(const int32_t* st, const int32_t* hist, const float* probs, int n, double c_puct,
                           double* pucts_out) {
    const int32_t total = st[20];
    return puct_choose_med(st, total >= 10 ? hist_median(hist, total) : 0.0, probs, n, c_puct, pucts_out);
}

// Categorical(probs).sample() with u from Philox: the first k whose
// running sum of the float32 softmax exceeds u
__device__ __forceinline__ int sample_softmax(const float* x, int n, float u) {
    float m = x[0];
    for (int k = 1; k < n; k++) m = fmaxf(m, x[k]);
    float sum = 0.f;
    for (int k = 0; k < n; k++) sum += __expf(x[k] - m);
    const float target = u * sum;
    float acc = 0.f;
    for (int k = 0; k < n - 1; k++) {
        acc += __expf(x[k] - m);
        if (acc > target) return k;
    }
    return n - 1;
}

// one candidate's logit: f32, or bf16 (the padded head GEMM's output), `ls` apart
template <bool LB>
__device__ __forceinline__ float logit_at(const void* lg, int64_t i, int ls) {
    if constexpr (LB) {
        const uint32_t u = (uint32_t)((const uint16_t*)lg)[i * ls] << 16;
        return __uint_as_float(u);
    } else {
        return ((const float*)lg)[i * ls];
    }
}

// Categorical(softmax(x[0..n))).sample() over a register row (unrolled to 10)
__device__ __forceinline__ int sample_row(const float (&x)[kHand], int n, float u) {
    float m = x[0];
#pragma unroll
    for (int k = 1; k < kHand; k++) m = (k < n) ? fmaxf(m, x[k]) : m;
    float e[kHand], sum = 0.f;
#pragma unroll
    for (int k = 0; k < kHand; k++) {
        e[k] = (k < n) ? __expf(x[k] - m) : 0.f;
        sum += e[k];
    }
    const float target = u * sum;
    float acc = 0.f;
    int pick = n - 1;
#pragma unroll
    for (int k = 0; k < kHand - 1; k++) {
        acc += e[k];
        pick = (k < n - 1 && acc > target && pick == n - 1 && k < pick) ? k : pick;
    }
    return pick;
}

template <int N, bool LB>
__global__ void k_puct_step(DevState s, PuctArgs a, const void* logits, int ls, int t, int n_cur) {
    const int64_t d = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (d >= a.D) return;
    int64_t g;
    int p;
    dec_to_gp(a, d, g, p);
    int32_t* ro = a.ro + d * kRoWords;
    Game<N> G;
#pragma unroll
    for (int q = 0; q < N; q++) G.hand[q] = ro_hand(ro, q);
    G.b = ro_board(ro);
    const uint64_t gid = s.game_offset + (uint64_t)g;
    const uint64_t stream = ((uint64_t)(uint32_t)gid << 32) | ((uint64_t)p << 28) | ((uint64_t)a.rollout << 8) | (uint64_t)(1 + t);
    uint32_t card[N], pen[N];
    int first = ro[41];
    const int kp = players_of(a, g);
    // every seat's logits first: N x n_cur independent loads in flight
    float lg[N][kHand];
#pragma unroll
    for (int q = 0; q < N; q++)
#pragma unroll
        for (int k = 0; k < kHand; k++)
            lg[q][k] = (q < kp && k < n_cur) ? logit_at<LB>(logits, (d * N + q) * n_cur + k, ls) : 0.f;
#pragma unroll
    for (int q = 0; q < N; q++) {
        if (q >= kp) {  // absent seat of a smaller tournament game
            card[q] = 0xFFu;
            continue;
        }
        int idx;
        if (t == 0 && q == 0 && (a.flags & 1)) {
            idx = puct_choose(a.stats + d * kStatWords, a.hist + d * kHistBins, a.root_probs + d * kHand, n_cur,
                              a.c_puct, nullptr);
        } else {
            idx = sample_row(lg[q], n_cur, philox_uniform(a.seed_lo ^ puct_step_of(a), a.seed_hi, stream, (uint32_t)q));
        }
        if (t == 0 && q == 0) first = idx;
        card[q] = hand_get(G.hand[q], (uint32_t)idx);
        hand_del(G.hand[q], (uint32_t)idx);
    }
    resolve<N, true>(G.b, card, pen);
    const int32_t outcome = ro[40] - (int32_t)pen[0];
    if (n_cur == 1) {
        // backup: outcomes[first].append(outcome) (mcts.py:100)
        int32_t* st = a.stats + d * kStatWords;
        st[first] += outcome;
        st[10 + first] += 1;
        st[20] += 1;
        st[21] = (st[20] == 1) ? outcome : min(st[21], outcome);
        st[22] = (st[20] == 1) ? outcome : max(st[22], outcome);
        a.hist[d * kHistBins + (outcome + 171)] += 1;
    } else {
        ro[0] = G.b.lo.x, ro[1] = G.b.lo.y, ro[2] = G.b.lo.z, ro[3] = G.b.lo.w;
        ro[4] = G.b.hi.x, ro[5] = G.b.hi.y, ro[6] = G.b.hi.z, ro[7] = G.b.hi.w;
#pragma unroll
        for (int q = 0; q < N; q++) {
            ro[8 + 3 * q] = (int32_t)(uint32_t)G.hand[q].lo;
            ro[9 + 3 * q] = (int32_t)(uint32_t)(G.hand[q].lo >> 32);
            ro[10 + 3 * q] = (int32_t)G.hand[q].hi;
        }
        ro[40] = outcome;
        ro[41] = first;
    }
}

// The same step with one lane per SEAT (L lanes per decision, L = N rounded
// up to a power of two, L <= 8): each lane loads its seat's hand and logits,
// draws its card (the same Philox uniform, counter = seat, as k_puct_step)
// and stores its hand back; the decision's first lane gathers the cards
// (lane shuffles), resolves, and writes the board / outcome / backup.  L
// times the lanes of k_puct_step (D = 8192 x 4 decisions: 2 waves per SIMD
// instead of half a wave), the per-decision latency chain split over them.
// lane i of the step (seat i & (L - 1) of decision i / L); logit(dd, q, k):
// candidate k's logit of seat q of decision dd; info(dd, g, p, kp): its game, seat and the
// game's players (dec_info from the decision list / tournament seats, or a cached copy)
struct DecInfo {
    __device__ __forceinline__ void operator()(const PuctArgs& a, int64_t dd, int64_t& g, int& p, int& kp) const {
        dec_to_gp(a, dd, g, p);
        kp = players_of(a, g);
    }
};

template <int N, int L, class Logit, class Info = DecInfo>
__device__ __forceinline__ void step_seat(const DevState& s, const PuctArgs& a, Logit logit, int t, int n_cur,
                                          int64_t i, int64_t d_hi = -1, int64_t d_dead = -1, Info info = Info{}) {
    const int64_t d = i / L;
    const int q = (int)(i & (L - 1));
    // lanes past the last decision (or past d_hi, with d_dead a decision they may read) follow along
    // (shuffles) and write nothing
    const bool live = d < a.D && (d_hi < 0 || d < d_hi);
    const int64_t dd = live ? d : (d_dead >= 0 ? d_dead : a.D - 1);
    int64_t g;
    int p, kp;
    info(a, dd, g, p, kp);
    int32_t* ro = a.ro + dd * kRoWords;
    const bool seat = q < N && q < kp;
    // the resolving lane's words, loaded with the seat's (no second round trip after the shuffles;
    // nothing below writes them before the resolve)
    Board b{};
    int32_t r40 = 0, r41 = 0, s20 = 0, s21 = 0, s22 = 0, sf = 0, cf = 0;
    if (q == 0) {
        b = ro_board(ro);
        r40 = ro[40], r41 = ro[41];
        if (n_cur == 1) {
            const int32_t* st = a.stats + dd * kStatWords;
            s20 = st[20], s21 = st[21], s22 = st[22];
            if (t > 0) sf = st[r41], cf = st[10 + r41];  // the backed-up move's words (first = r41 past t = 0)
        }
    }
    uint32_t card = 0xFFu;
    int idx = 0;
    const int lead_lane = (int)(threadIdx.x & 63) & ~(L - 1);
    int root_idx = 0;
    if (t == 0 && (a.flags & 1)) {  // the root PUCT choice: every lane of the decision scores a part
        const int32_t total = a.stats[dd * kStatWords + 20];
        double med = __builtin_nan("");
        if (total >= 10) med = hist_median_lanes<L>(a.hist + dd * kHistBins, total, q, lead_lane);
        root_idx = puct_choose_lanes<L>(a.stats + dd * kStatWords, med, a.root_probs + dd * kHand, n_cur, a.c_puct, q,
                                        lead_lane);
    }
    if (seat) {
        float lg[kHand];
#pragma unroll
        for (int k = 0; k < kHand; k++) lg[k] = (k < n_cur) ? logit(dd, q, k) : 0.f;
        Hand h = ro_hand(ro, q);
        if (t == 0 && q == 0 && (a.flags & 1)) {
            idx = root_idx;
        } else {
            const uint64_t gid = s.game_offset + (uint64_t)g;
            const uint64_t stream =
                ((uint64_t)(uint32_t)gid << 32) | ((uint64_t)p << 28) | ((uint64_t)a.rollout << 8) | (uint64_t)(1 + t);
            idx = sample_row(lg, n_cur, philox_uniform(a.seed_lo ^ puct_step_of(a), a.seed_hi, stream, (uint32_t)q));
        }
        card = hand_get(h, (uint32_t)idx);
        hand_del(h, (uint32_t)idx);
        if (n_cur > 1 && live) {
            ro[8 + 3 * q] = (int32_t)(uint32_t)h.lo;
            ro[9 + 3 * q] = (int32_t)(uint32_t)(h.lo >> 32);
            ro[10 + 3 * q] = (int32_t)h.hi;
        }
    }
    // the decision's cards to its first lane (absent seats: 0xFF, resolve skips them)
    const int lead = (int)(threadIdx.x & 63) & ~(L - 1);
    uint32_t cards[N];
#pragma unroll
    for (int r = 0; r < N; r++) cards[r] = (uint32_t)__shfl((int)card, lead + r);
    const int first_idx = __shfl(idx, lead);
    if (q != 0 || !live) return;
    uint32_t pen[N];
    resolve<N, true>(b, cards, pen);
    const int first = (t == 0) ? first_idx : r41;
    const int32_t outcome = r40 - (int32_t)pen[0];
    if (n_cur == 1) {
        int32_t* st = a.stats + dd * kStatWords;
        if (t > 0) {
            st[first] = sf + outcome;
            st[10 + first] = cf + 1;
        } else {
            st[first] += outcome;
            st[10 + first] += 1;
        }
        const int32_t total = s20 + 1;
        st[20] = total;
        st[21] = (total == 1) ? outcome : min(s21, outcome);
        st[22] = (total == 1) ? outcome : max(s22, outcome);
        a.hist[dd * kHistBins + (outcome + 171)] += 1;
    } else {
        ro[0] = b.lo.x, ro[1] = b.lo.y, ro[2] = b.lo.z, ro[3] = b.lo.w;
        ro[4] = b.hi.x, ro[5] = b.hi.y, ro[6] = b.hi.z, ro[7] = b.hi.w;
        ro[40] = outcome;
        ro[41] = first;
    }
}

template <int N, int L, bool LB>
__global__ void k_puct_step_seats(DevState s, PuctArgs a, const void* logits, int ls, int t, int n_cur) {
    step_seat<N, L>(
        s, a, [&](int64_t dd, int q, int k) { return logit_at<LB>(logits, (dd * N + q) * n_cur + k, ls); }, t, n_cur,
        (int64_t)blockIdx.x * blockDim.x + threadIdx.x);
}

// ---- the whole rollout MLP in one kernel (sn_puct_mlp_seats) -------------
// A workgroup loads W1s / W2 into LDS once and then loops over groups of 64
// consecutive rollout seats (persistent grid: two workgroups per CU, the
// occupancy the 64-row MFMA tiles' registers allow).  Per group: phase 1
// builds the seats' [0, obs, 1] rows in LDS (the features of write_row,
// four lanes per seat) and the candidates' card
// features, phase 2 computes base = W1s . rows for the 64 seats with MFMA
// (layer 1's obs part, K = 64) into LDS (bf16, as the PyTorch GEMM rounds
// it), phase 3 runs mlp_tile over the group's rows reading base and the
// cards from LDS.  (The round-4 GEMM form -- seat rows + a PyTorch GEMM +
// a tile kernel, two launches and the [S][56] / [S][112] HBM round trips --
// and the round-5 per-candidate layer-1 form measured slower and were
// removed in round 6)
constexpr int kSeatBlock = 64;
constexpr int kSeatRowK = 64;               // seat-row features (48 + the ones feature, zero-padded)
constexpr int kSeatRowLds = kSeatRowK + 8;  // LDS stride (144 B)
constexpr int kBaseLds = kMlpK + 8;         // 120 bf16 (240 B) per seat of base in LDS

__device__ __forceinline__ uint16_t bf16_bits(float v) { return __builtin_bit_cast(uint16_t, __float2bfloat16(v)); }

// phase 1, lane `part` (0..3) of seat `sl`: hand features / cards k = part,
// part + 4, part + 8, board row `part`, a quarter of the zero padding, and
// one of the constant features (write_row's values, feature 0 = the card
// slot left 0: the candidates' cards enter through w1c)
// what lane `part` of seat i reads from the rollout state (global loads,
// issued one group ahead by k_puct_mlp_seats)
struct SeatIn {
    uint32_t h0, h1, h2;  // the seat's hand words (ro_hand)
    uint32_t lo, hi;      // board row `part` (ro_board)
    int kp;               // players of the seat's game
    bool live;            // a seated player (q < kp)
};

// the same for seat q of decision d whose game seats kp players (known)
__device__ __forceinline__ SeatIn seat_load_kp(const PuctArgs& a, int64_t d, int q, int kp, int part) {
    const int32_t* ro = a.ro + d * kRoWords;
    SeatIn in;
    in.kp = kp;
    in.live = q < kp;
    const int qq = in.live ? q : 0;
    in.h0 = (uint32_t)ro[8 + 3 * qq], in.h1 = (uint32_t)ro[9 + 3 * qq], in.h2 = (uint32_t)ro[10 + 3 * qq];
    in.lo = (uint32_t)ro[part], in.hi = (uint32_t)ro[4 + part];
    return in;
}

__device__ __forceinline__ SeatIn seat_load(const PuctArgs& a, int N, int64_t i, int part) {
    const int64_t d = i / N;
    const int q = (int)(i - d * N);
    const int32_t* ro = a.ro + d * kRoWords;
    SeatIn in;
    in.kp = N;
    if (a.lgs) {
        int64_t g;
        int p;
        dec_to_gp(a, d, g, p);
        in.kp = players_of(a, g);
    }
    in.live = q < in.kp;
    const int qq = in.live ? q : 0;
    in.h0 = (uint32_t)ro[8 + 3 * qq], in.h1 = (uint32_t)ro[9 + 3 * qq], in.h2 = (uint32_t)ro[10 + 3 * qq];
    in.lo = (uint32_t)ro[part], in.hi = (uint32_t)ro[4 + part];
    return in;
}

// the row features as bf16 bits by value (write_row's nrm + rounding, looked
// up instead of a correctly rounded f32 division per feature): card / hand
// slot c in -1..103 at [c + 1], row length, bull heads and player count after
constexpr int kLutCard = 0, kLutLen = 105, kLutHeads = 113, kLutN = 177, kLutSize = 193;
__device__ __forceinline__ void build_row_lut(uint16_t* lut) {
    for (int i = threadIdx.x; i < kLutSize; i += blockDim.x) {
        float v;
        if (i < kLutLen) v = nrm((float)(i - 1), 0.f, 103.f);
        else if (i < kLutHeads) v = nrm((float)(i - kLutLen), 1.f, 5.f);
        else if (i < kLutN) v = nrm((float)(i - kLutHeads), 1.f, 10.f);
        else v = nrm((float)(i - kLutN), 0.f, 6.f);
        lut[i] = bf16_bits(v);
    }
}

__device__ __forceinline__ void seat_row_part(const SeatIn& in, int n_cur, int part, uint16_t* row, float* cd,
                                              const uint16_t* lut) {
    const bool live = in.live;
    const int kp = in.kp;
    Hand h;
    h.lo = in.h0 | ((uint64_t)in.h1 << 32);
    h.hi = in.h2;
    auto card_bits = [&](uint32_t c) { return lut[kLutCard + (c == 0xFFu ? 0u : min(c, 103u) + 1u)]; };  // 0xFF: -1
    // every table lookup first, then the row writes: the LDS reads in flight together (written
    // interleaved, each write waited for its own read)
    uint16_t hb[3], rc[kThreshold];
#pragma unroll
    for (int j = 0; j < 3; j++) {
        const int k = part + 4 * j;
        hb[j] = (k < kHand) ? card_bits(hand_get(h, (uint32_t)(k < kHand ? k : 0))) : (uint16_t)0;
    }
    const uint32_t lo = in.lo, hi = in.hi;
    const uint32_t len = len_of(hi);
    const uint16_t lenb = lut[kLutLen + min(len, 7u)];
    const uint16_t endb = card_bits(end_of(hi));
    const uint16_t headb = lut[kLutHeads + min(heads_in(hi), 63u)];  // <= 35 in a game
#pragma unroll
    for (int c = 0; c < kThreshold; c++) {
        const uint32_t v = (c < 5 && (uint32_t)c < len) ? card_at(lo, hi, c < 5 ? c : 0) : 0xFFu;
        rc[c] = card_bits(v);
    }
    const uint16_t kpb = lut[kLutN + min(kp, 15)];
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int j = 0; j < 3; j++) {
        const int k = part + 4 * j;
        if (k < kHand) {
            row[1 + k] = live ? hb[j] : (uint16_t)0;
            cd[k] = (live && k < n_cur) ? __uint_as_float((uint32_t)hb[j] << 16) : 0.f;
        }
    }
    row[12 + part] = live ? lenb : (uint16_t)0;
    row[16 + part] = live ? endb : (uint16_t)0;
    row[20 + part] = live ? headb : (uint16_t)0;
#pragma unroll
    for (int c = 0; c < kThreshold; c++) row[24 + part * kThreshold + c] = live ? rc[c] : (uint16_t)0;
#pragma unroll
    for (int j = 0; j < 4; j++) {
        const int f = kRowLen + 1 + part + 4 * j;
        if (f < kSeatRowK) row[f] = 0;
    }
    if (part == 0) row[0] = 0;
    if (part == 1) row[11] = live ? kpb : (uint16_t)0;
    if (part == 2) row[kRowLen] = bf16_bits(1.f);
}

__global__ __launch_bounds__(256, 2) void k_puct_mlp_seats(PuctArgs a, int N, int n_cur, const uint16_t* w1s,
                                                          const float* w1c, const uint16_t* w2, const float* head,
                                                          float* logits) {
    constexpr int TNT = 2;  // 32-row halves per phase-3 tile (32-row tiles measured slower)
    constexpr int kWaves = kBlock / 64;
    __shared__ __attribute__((aligned(16))) uint16_t sW[kMlpM * kMlpLdsK];            // W2 [128][120]
    __shared__ __attribute__((aligned(16))) uint16_t sRow[kSeatBlock * kSeatRowLds];  // seat rows [64][72]
    __shared__ __attribute__((aligned(16))) uint16_t sBase[2][kSeatBlock * kBaseLds];  // base [64][120], 2 groups
    __shared__ __attribute__((aligned(16))) float sCard[2][kSeatBlock * kHand];
    __shared__ __attribute__((aligned(16))) float sC[kMlpK];
    __shared__ __attribute__((aligned(16))) uint32_t sH2[kMlpM / 2];
    __shared__ uint16_t sLut[kLutSize];
    const int tid = threadIdx.x;
    const int wave = tid >> 6, lane = tid & 63, col = lane & 31, half = lane >> 5;
    build_row_lut(sLut);
    const int64_t S = a.D * N;
    const int64_t groups = (S + kSeatBlock - 1) / kSeatBlock;
    for (int i = tid; i < kMlpM * (kMlpK / 8); i += blockDim.x) {
        const int o = i / (kMlpK / 8), c = i - o * (kMlpK / 8);
        *(uint4*)&sW[o * kMlpLdsK + 8 * c] = *(const uint4*)&w2[o * kMlpK + 8 * c];
    }
    for (int i = tid; i < kMlpK; i += blockDim.x) sC[i] = w1c[i];
    load_head_pairs(head, sH2);
    // phase 2's A fragments (W1s rows 32 wave + col, the four k-steps) stay in registers
    bf16x8_t w1f[kSeatRowK / 16];
#pragma unroll
    for (int ks = 0; ks < kSeatRowK / 16; ks++)
        w1f[ks] = __builtin_bit_cast(bf16x8_t, *(const uint4*)&w1s[(32 * wave + col) * kSeatRowK + 16 * ks + 8 * half]);
    const int sl = tid >> 2, part = tid & 3;  // phase 1: four lanes per seat
    auto group_load = [&](int64_t grp) {
        const int64_t s0 = grp * kSeatBlock;
        return seat_load(a, N, s0 + min<int64_t>(sl, S - s0 - 1), part);
    };
    // one 64-row phase-3 tile of a group held in buffer `buf`
    auto run_tile = [&](int buf, uint32_t tile, uint32_t rows, uint32_t rbase) {
        uint32_t rr[TNT];
        float x[TNT];
        const uint16_t* brow[TNT];
#pragma unroll
        for (int nt = 0; nt < TNT; nt++) {
            rr[nt] = tile * 32u * TNT + 32u * nt + (uint32_t)col;  // group-local row
            const uint32_t rc = rr[nt] < rows ? rr[nt] : rows - 1u;
            const uint32_t q = rc / (uint32_t)n_cur;
            x[nt] = sCard[buf][q * kHand + (rc - q * (uint32_t)n_cur)];
            brow[nt] = sBase[buf] + q * kBaseLds;
        }
        float out[TNT];
        mlp_tile<TNT>(brow, x, sW, sC, sH2, col, half, out);
#pragma unroll
        for (int nt = 0; nt < TNT; nt++)
            if (half == 0 && rr[nt] < rows) logits[rbase + rr[nt]] = out[nt];
    };
    // tiles of the previous group left for this iteration (the waves share a
    // tile list of those + this group's tiles; up to 3 of this group's are
    // carried to the next iteration so that every wave gets the same count)
    uint32_t pend_first = 0u, pend_cnt = 0u, pend_rows = 0u, pend_rbase = 0u;
    SeatIn nxt = group_load(min<int64_t>(blockIdx.x, groups - 1));
    int it = 0;
    for (int64_t grp = blockIdx.x; grp < groups; grp += gridDim.x, it++) {
    const int buf = it & 1;
    const int64_t s0 = grp * kSeatBlock;
    const int nseat = (int)min<int64_t>(kSeatBlock, S - s0);
    const SeatIn cur = nxt;
    __syncthreads();  // the last iteration's tiles are done with this buffer, phase 2 with sRow
    // phase 1: the seats' rows and card features
    seat_row_part(cur, n_cur, part, sRow + sl * kSeatRowLds, sCard[buf] + sl * kHand, sLut);
    __syncthreads();
    // phase 2: base[seat][j] = sum_k W1s[j][k] rows[seat][k]; wave w: outputs j in [32w, 32w + 32)
    {
        f32x16_t acc[2];
#pragma unroll
        for (int ks = 0; ks < kSeatRowK / 16; ks++) {
            const int k0 = 16 * ks + 8 * half;
#pragma unroll
            for (int nt = 0; nt < 2; nt++) {
                const bf16x8_t bfr = __builtin_bit_cast(bf16x8_t, *(const uint4*)&sRow[(32 * nt + col) * kSeatRowLds + k0]);
                const f32x16_t zero = {};
                acc[nt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w1f[ks], bfr, ks ? acc[nt] : zero, 0, 0, 0);
            }
        }
#pragma unroll
        for (int nt = 0; nt < 2; nt++)
#pragma unroll
            for (int r = 0; r < 16; r += 2) {  // C rows j, j + 1 (r & 3 in {0, 1} or {2, 3}): one b32 store
                const int j = 32 * wave + (r & 3) + 8 * (r >> 2) + 4 * half;
                if (j < kMlpK)
                    *(uint32_t*)&sBase[buf][(32 * nt + col) * kBaseLds + j] = pack_bf16(acc[nt][r], acc[nt][r + 1]);
            }
    }
    __syncthreads();
    const bool more = grp + gridDim.x < groups;
    // the next group's rollout-state loads fly during phase 3
    if (more) nxt = group_load(grp + gridDim.x);
    // phase 3: the shared tile list
    const uint32_t rows = (uint32_t)nseat * (uint32_t)n_cur;
    const uint32_t tiles = (rows + 32u * TNT - 1u) / (32u * TNT);
    const uint32_t rbase = (uint32_t)s0 * (uint32_t)n_cur;
    const uint32_t total = pend_cnt + tiles;
    uint32_t defer = more ? total % kWaves : 0u;
    if (defer > tiles) defer = 0u;  // only this group's tiles can wait
    for (uint32_t i = (uint32_t)wave; i < total - defer; i += kWaves) {
        if (i < pend_cnt) run_tile(buf ^ 1, pend_first + i, pend_rows, pend_rbase);
        else run_tile(buf, i - pend_cnt, rows, rbase);
    }
    pend_first = tiles - defer, pend_cnt = defer, pend_rows = rows, pend_rbase = rbase;
    }
}

// ---- whole rollouts in one kernel (sn_puct_rollouts) ----------------------
// Every rollout step of k_puct_mlp_seats + k_puct_step_seats touches one
// decision's rollout state, its seats' logits and its statistics only, so
// ONE WAVE can carry a group of 64 / L decisions (their <= 64 seat rows, L
// lanes per decision) through whole rollouts -- every step of rollouts
// r0 .. r0 + nr - 1, in order, rollout r's first move chosen by PUCT from
// the statistics rollouts < r backed up -- with no other wave involved and
// no barrier: per step the seats' rows (phase 1, a lane per seat), the
// per-seat layer-1 MFMA (phase 2: 4 output tiles x 2 seat halves x 4
// k-steps), the candidates' 64-row tiles (phase 3, mlp_tile) into logits in
// LDS, then step_seat on them.  The same code, the same values as the
// two-launches-per-step loop.  A workgroup of four waves shares W2 in LDS
// (one workgroup per CU: four groups in flight per CU, each wave's MFMA
// chain keeping its SIMD busy), each wave has its own rows / base / cards /
// logits / rollout states.  (The first form -- a workgroup per group, four
// barriers per step -- ran 12 us per group-step: two groups in flight per
// CU, slower than the launch-per-step loop.)  Rollout r's initial states
// are ro_base + (r - r0) * D * kRoWords (sn_puct_deal_batch dealt them); the
// wave's copy in LDS is the one the steps read and write.
constexpr int kRollSeats = 32;  // seats per wave's group (32 / L... 64 / L / 2 decisions)
constexpr int kRollWaveLds = kRollSeats * kSeatRowLds * 2 + kRollSeats * kBaseLds * 2 + kRollSeats * kHand * 4 +
                             8 * kRoWords * 4 + 8 * 2 * 4;  // rows (aliased by logits) + base + cards + states +
                                                            // the decisions' game / seat / players: 15 168 B

// k_puct_rollouts phase profiler (diagnostics, -DSECHS_PHASE_PROF builds only,
// sn_debug_puct_phases): shader-clock cycles per wave in the state copy-in,
// the seat rows (phase 1), the per-seat layer-1 MFMA (phase 2), the
// candidate tiles (phase 3), the step (t > 0) and the first step (t = 0: the
// PUCT root choice); [7] counts waves
enum { RP_COPY = 0, RP_ROWS, RP_BASE, RP_TILES, RP_STEP, RP_STEP0, RP_N };  // RP_STEP0: the t = 0 step (PUCT choice)
#ifdef SECHS_PHASE_PROF
__device__ unsigned long long g_puct_phase[8];
struct RollProf {
    uint64_t t, acc[RP_N];
    __device__ __forceinline__ void start() {
        t = __builtin_readcyclecounter();
        for (int k = 0; k < RP_N; k++) acc[k] = 0ull;
    }
    __device__ __forceinline__ void mark(int k) {
        const uint64_t n = __builtin_readcyclecounter();
        acc[k] += n - t;
        t = n;
    }
    __device__ __forceinline__ void flush(int lane) {
        if (lane == 0) {
            for (int k = 0; k < RP_N; k++) atomicAdd(&g_puct_phase[k], (unsigned long long)acc[k]);
            atomicAdd(&g_puct_phase[7], 1ull);
        }
    }
};
#else
struct RollProf {
    __device__ __forceinline__ void start() {}
    __device__ __forceinline__ void mark(int) {}
    __device__ __forceinline__ void flush(int) {}
};
#endif

// sn_puct_mlp_seats' arithmetic.
template <int N, int L>
__global__ __launch_bounds__(512, 1) void k_puct_rollouts(DevState s, PuctArgs a, int r0, int nr, int32_t* ro_base,
                                                         const uint16_t* w1s, const float* w1c, const uint16_t* w2,
                                                         const float* head, int DG) {
    constexpr int TNT = 2;
    constexpr int kWaves = 512 / 64;  // two per SIMD
    // DG: decisions per group (<= kRollSeats / L; the host picks the fewest that keep the
    // rounds of groups over the grid's waves at their minimum)
    static_assert(kRollSeats / L <= 8 && (kRollSeats / L) * N <= kRollSeats, "a group's seats and states fit");
    constexpr int kWld = kMlpLdsK, kWk = kMlpK;
    __shared__ __attribute__((aligned(16))) uint16_t sW[kMlpM * kWld];  // W2 [128][120], shared
    __shared__ __attribute__((aligned(16))) float sC[kMlpK];
    __shared__ __attribute__((aligned(16))) uint32_t sH2[kMlpM / 2];
    __shared__ uint16_t sLut[kLutSize];
    __shared__ __attribute__((aligned(16))) uint8_t sWave[kWaves][kRollWaveLds];
    const int tid = threadIdx.x;
    const int wave = tid >> 6, lane = tid & 63, col = lane & 31, half = lane >> 5;
    build_row_lut(sLut);
    for (int i = tid; i < kMlpM * (kWk / 8); i += blockDim.x) {
        const int o = i / (kWk / 8), c = i - o * (kWk / 8);
        *(uint4*)&sW[o * kWld + 8 * c] = *(const uint4*)&w2[o * kWk + 8 * c];
    }
    for (int i = tid; i < kMlpK; i += blockDim.x) sC[i] = w1c[i];
    load_head_pairs(head, sH2);
    __syncthreads();  // the only barrier: the waves run independently from here
    uint16_t* sRow = (uint16_t*)sWave[wave];                 // [32][72]
    uint16_t* sBase = sRow + kRollSeats * kSeatRowLds;       // [32][120]
    // [32 x 10]: over sRow once phase 2 is done with it
    float* sLogit = (float*)sWave[wave];
    float* sCard = (float*)(sBase + kRollSeats * kBaseLds);  // [32][10]
    int32_t* sRo = (int32_t*)(sCard + kRollSeats * kHand);   // [DG][48]
    int32_t* sInf = sRo + 8 * kRoWords;                       // [DG][2]: game, seat | players << 8
    const int64_t groups = (a.D + DG - 1) / DG;
    auto fence = [] { __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront"); };
    const int sl = lane & (kRollSeats - 1), p0 = lane >> 5;  // phase 1: seat sl, parts p0 and p0 + 2
    RollProf pf;
    pf.start();
    for (int64_t grp = (int64_t)blockIdx.x * kWaves + wave; grp < groups; grp += (int64_t)gridDim.x * kWaves) {
        const int64_t d0 = grp * DG;
        const int nd = (int)min<int64_t>(DG, a.D - d0);
        const int nseat = nd * N;
        // the decisions' game, seat and players (a tournament's decision list and seat words: global loads
        // once per group instead of per step and lane)
        if (lane < DG) {
            int64_t g;
            int p, kp;
            DecInfo{}(a, d0 + min(lane, nd - 1), g, p, kp);
            sInf[2 * lane] = (int32_t)g, sInf[2 * lane + 1] = p | (kp << 8);
        }
        fence();
        auto info = [&](const PuctArgs&, int64_t dd, int64_t& g, int& p, int& kp) {
            const int j = (int)(dd - d0);
            g = sInf[2 * j];
            const int w = sInf[2 * j + 1];
            p = w & 255, kp = w >> 8;
        };
        for (int r = r0; r < r0 + nr; r++) {
            PuctArgs ar = a;
            ar.rollout = (uint32_t)r;
            {
                const int32_t* src = ro_base + ((int64_t)(r - r0) * a.D + d0) * kRoWords;
                for (int i = lane; i < nd * kRoWords; i += 64) sRo[i] = src[i];
            }
            ar.ro = sRo - d0 * kRoWords;
            fence();
            pf.mark(RP_COPY);
            for (int t = 0; t < a.n; t++) {
                const int m = a.n - t;
                // phase 1: two lanes per seat (rows past the group's seats repeat its last)
#pragma unroll
                for (int pp = 0; pp < 2; pp++) {
                    const int part = p0 + 2 * pp;
                    const int si = min(sl, nseat - 1), dj = si / N;
                    const SeatIn in = seat_load_kp(ar, d0 + dj, si - dj * N, sInf[2 * dj + 1] >> 8, part);
                    seat_row_part(in, m, part, sRow + sl * kSeatRowLds, sCard + sl * kHand, sLut);
                }
                fence();
                pf.mark(RP_ROWS);
                // phase 2: base[seat][j] = sum_k W1s[j][k] rows[seat][k] (one 32-seat tile)
                {
                    // the A fragments (W1s rows 32 mt + col) from L1 / L2 per step: held across phase 3
                    // they would spill (two waves per SIMD: 256 registers each)
                    bf16x8_t w1f[4][kSeatRowK / 16];
#pragma unroll
                    for (int mt = 0; mt < 4; mt++)
#pragma unroll
                        for (int ks = 0; ks < kSeatRowK / 16; ks++)
                            w1f[mt][ks] = __builtin_bit_cast(
                                bf16x8_t, *(const uint4*)&w1s[(32 * mt + col) * kSeatRowK + 16 * ks + 8 * half]);
                    f32x16_t acc[4];
#pragma unroll
                    for (int ks = 0; ks < kSeatRowK / 16; ks++) {
                        const bf16x8_t bfr =
                            __builtin_bit_cast(bf16x8_t, *(const uint4*)&sRow[col * kSeatRowLds + 16 * ks + 8 * half]);
                        const f32x16_t zero = {};
#pragma unroll
                        for (int mt = 0; mt < 4; mt++)
                            acc[mt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w1f[mt][ks], bfr, ks ? acc[mt] : zero, 0, 0, 0);
                    }
#pragma unroll
                    for (int mt = 0; mt < 4; mt++)
#pragma unroll
                        for (int rr = 0; rr < 16; rr += 2) {
                            const int j = 32 * mt + (rr & 3) + 8 * (rr >> 2) + 4 * half;
                            if (j < kMlpK)
                                *(uint32_t*)&sBase[col * kBaseLds + j] = pack_bf16(acc[mt][rr], acc[mt][rr + 1]);
                        }
                }
                fence();
                pf.mark(RP_BASE);
                // phase 3: the group's candidate rows, 64 per tile, logits to LDS (over the dead rows);
                // a last tile of <= 32 rows as one 32-row half (odd n_cur: half the MFMAs and B fragments)
                const uint32_t rows = (uint32_t)nseat * (uint32_t)m;
                auto run_tile = [&](auto tnt, uint32_t base) {
                    constexpr int T = decltype(tnt)::value;
                    uint32_t rw[T];
                    float x[T];
                    const uint16_t* brow[T];
#pragma unroll
                    for (int nt = 0; nt < T; nt++) {
                        rw[nt] = base + 32u * nt + (uint32_t)col;
                        const uint32_t rc = rw[nt] < rows ? rw[nt] : rows - 1u;
                        const uint32_t q = rc / (uint32_t)m;
                        x[nt] = sCard[q * kHand + (rc - q * (uint32_t)m)];
                        brow[nt] = sBase + q * kBaseLds;
                    }
                    float out[T];
                    mlp_tile<T>(brow, x, sW, sC, sH2, col, half, out);
                    if (base == 0u) fence();  // every lane's phase-2 row reads are done before logits land on them
#pragma unroll
                    for (int nt = 0; nt < T; nt++)
                        if (half == 0 && rw[nt] < rows) sLogit[rw[nt]] = out[nt];
                };
                const uint32_t full = rows / (32u * TNT), rest = rows - full * 32u * TNT;
                for (uint32_t tile = 0; tile < full; tile++) run_tile(std::integral_constant<int, TNT>{}, tile * 32u * TNT);
                if (rest > 32u) run_tile(std::integral_constant<int, TNT>{}, full * 32u * TNT);
                else if (rest) run_tile(std::integral_constant<int, 1>{}, full * 32u * TNT);
                fence();
                pf.mark(RP_TILES);
                // the step: L lanes per decision (step_seat, as k_puct_step_seats); lanes past the
                // group's DG decisions (the upper half of the wave) follow along and write nothing
                step_seat<N, L>(
                    s, ar, [&](int64_t dd, int q, int k) { return sLogit[((dd - d0) * N + q) * m + k]; }, t, m,
                    d0 * L + lane, d0 + nd, d0, info);
                fence();
                pf.mark(t == 0 ? RP_STEP0 : RP_STEP);
            }
        }
    }
    pf.flush(lane);
}

// _choose_action_from_outcomes (mcts.py:156-165, temperature None): best mean
// over moves with playouts, strict '>'; one-card hands play it directly
__global__ void k_puct_choose(DevState s, PuctArgs a, int32_t* actions, int32_t* best_index) {
    const int64_t d = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (d >= a.D) return;
    int64_t g;
    int p;
    dec_to_gp(a, d, g, p);
    const Hand h = load_hand(s, p, g);
    int best = 0;
    if (a.n > 1) {
        const int32_t* st = a.stats + d * kStatWords;
        double bm = -__builtin_inf();
        for (int k = 0; k < a.n; k++) {
            if (st[10 + k] == 0) continue;
            const double m = (double)st[k] / (double)st[10 + k];
            if (m > bm) bm = m, best = k;
        }
    }
    actions[g * s.N + p] = (int32_t)hand_get(h, (uint32_t)best);
    if (best_index) best_index[d] = best;
}

// PUCTCustomedAgent (mcts.py:325-451): no rollouts; the 2-head net's value
// head picks the move (_choose_action_mc_func, mcts.py:385-395: the first
// argmax of the values over the legal list), its policy head gives the
// move's log-probability (Categorical(softmax(policy)).log_prob) and the
// chosen value is the step's "outcome".  heads = [D*n][2] f32 (policy, value)
// in sn_puct_root_rows order.  One lane per decision.
__global__ void k_pcv_choose(DevState s, PuctArgs a, const float* heads, int32_t* actions, int32_t* best_index,
                             float* log_prob, float* value) {
    const int64_t d = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (d >= a.D) return;
    int64_t g;
    int p;
    dec_to_gp(a, d, g, p);
    const Hand h = load_hand(s, p, g);
    const float2* x = (const float2*)heads + d * a.n;
    float bv = x[0].y, m = x[0].x;
    int best = 0;
    for (int k = 1; k < a.n; k++) {
        const float2 v = x[k];
        if (v.y > bv) bv = v.y, best = k;
        m = fmaxf(m, v.x);
    }
    float sum = 0.f;
    for (int k = 0; k < a.n; k++) sum += expf(x[k].x - m);
    actions[g * s.N + p] = (int32_t)hand_get(h, (uint32_t)best);
    if (best_index) best_index[d] = best;
    if (log_prob) log_prob[d] = (x[best].x - m) - logf(sum);
    if (value) value[d] = bv;
}

// BatchedReinforceAgent.forward (agents/policy.py:137-156) for every
// deciding seat: Categorical(softmax(logits)).sample() with a Philox uniform
// keyed (seed ^ step, game, seat; rollout tag 0xFFFFF, never a PUCT
// rollout's), plus log_prob and entropy of the distribution.  logits
// [D*n] f32 in sn_puct_root_rows order.  One lane per decision.
__global__ void k_policy_sample(DevState s, PuctArgs a, const float* logits, int32_t* actions, int32_t* index,
                                float* log_prob, float* entropy) {
    const int64_t d = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (d >= a.D) return;
    int64_t g;
    int p;
    dec_to_gp(a, d, g, p);
    const Hand h = load_hand(s, p, g);
    const float* x = logits + d * a.n;
    const uint64_t gid = s.game_offset + (uint64_t)g;
    const uint64_t stream = ((uint64_t)(uint32_t)gid << 32) | ((uint64_t)p << 28) | (0xFFFFFull << 8);
    const int k = sample_softmax(x, a.n, philox_uniform(a.seed_lo ^ puct_step_of(a), a.seed_hi, stream, 0u));
    float m = x[0];
    for (int j = 1; j < a.n; j++) m = fmaxf(m, x[j]);
    float sum = 0.f, sx = 0.f;
    for (int j = 0; j < a.n; j++) {
        const float e = expf(x[j] - m);
        sum += e;
        sx += e * (x[j] - m);
    }
    const float lse = logf(sum);
    actions[g * s.N + p] = (int32_t)hand_get(h, (uint32_t)k);
    if (index) index[d] = k;
    if (log_prob) log_prob[d] = (x[k] - m) - lse;
    if (entropy) entropy[d] = lse - sx / sum;  // -sum p log p
}

// test hook for the formula fixtures (F5): stats/hist/probs given per decision
__global__ void k_puct_score(int64_t D, int n_max, const int32_t* n, const int32_t* stats, const int32_t* hist,
                             const float* probs, double c_puct, double* pucts, int32_t* choice) {
    const int64_t d = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (d >= D) return;
    choice[d] = puct_choose(stats + d * kStatWords, hist + d * kHistBins, probs + d * kHand, n[d], c_puct,
                            pucts + d * kHand);
    (void)n_max;
}

// ============================================================================
// C ABI
// ============================================================================
static sn_status puct_args(sn_env* e, const sn_puct* q, PuctArgs& a) {
    if (!e || !q) return set_error(SN_EINVAL, "NULL argument");
    if (q->n < 1 || q->n > kHand) return set_error(SN_EINVAL, "hand size out of range");
    a.N = e->s.N;
    a.lgs = e->s.lg_K ? e->s.lgs : nullptr;
    if (q->dec_list) {
        if (q->num_dec < 1 || q->num_dec > e->s.B * e->s.N) return set_error(SN_EINVAL, "num_dec out of range");
        a.dec = q->dec_list;
        a.D = q->num_dec;
        a.M = 1u;
        a.seats_mask = 0u;
    } else {
        if (a.lgs) return set_error(SN_EINVAL, "a tournament handle's engines take decision lists (dec_list)");
        const uint32_t mask = q->seats_mask & ((1u << e->s.N) - 1u);
        if (!mask) return set_error(SN_EINVAL, "seats_mask selects no seat");
        a.M = (uint32_t)__builtin_popcount(mask);
        a.seats_mask = mask;
        a.D = e->s.B * a.M;
    }
    a.n = q->n;
    a.flags = q->puct_root ? 1 : 0;
    a.c_puct = q->c_puct;
    a.seed_lo = (uint32_t)q->seed, a.seed_hi = (uint32_t)(q->seed >> 32), a.step = q->step;
    a.rollout = q->rollout;
    a.step_dev = q->step_dev;
    a.avail = q->avail;
    a.ro = q->rollouts;
    a.stats = q->stats;
    a.hist = q->hist;
    a.root_probs = q->root_probs;
    return SN_OK;
}

extern "C" {

sn_status sn_puct_root_rows(sn_env* e, const sn_puct* q, void* rows, int bf16, void* stream) {
    PuctArgs a{};
    sn_status st = puct_args(e, q, a);
    if (st != SN_OK) return st;
    hipStream_t s = (hipStream_t)stream;
    if (bf16)
        hipLaunchKernelGGL(k_puct_root_rows<__hip_bfloat16>, dim3(grid_for(a.D * a.n)), dim3(kBlock), 0, s, e->s, a,
                           (__hip_bfloat16*)rows);
    else
        hipLaunchKernelGGL(k_puct_root_rows<float>, dim3(grid_for(a.D * a.n)), dim3(kBlock), 0, s, e->s, a, (float*)rows);
    HIP_TRY(hipGetLastError());
    return SN_OK;
}

sn_status sn_puct_init(sn_env* e, const sn_puct* q, const float* root_logits, void* stream) {
    PuctArgs a{};
    sn_status st = puct_args(e, q, a);
    if (st != SN_OK) return st;
    hipLaunchKernelGGL(k_puct_init, dim3(grid_for(a.D)), dim3(kBlock), 0, (hipStream_t)stream, a, root_logits);
    HIP_TRY(hipGetLastError());
    return SN_OK;
}

sn_status sn_puct_deal(sn_env* e, const sn_puct* q, void* stream) {
    PuctArgs a{};
    sn_status st = puct_args(e, q, a);
    if (st != SN_OK) return st;
    hipStream_t s = (hipStream_t)stream;
    SN_DISPATCH_N(e->s.N, hipLaunchKernelGGL((k_puct_deal<NN>), dim3(grid_for(a.D)), dim3(kBlock), 0, s, e->s, a));
    HIP_TRY(hipGetLastError());
    return SN_OK;
}

sn_status sn_puct_deal_batch(sn_env* e, const sn_puct* q, int r0, int nr, void* ro_out, void* stream) {
    PuctArgs a{};
    sn_status st = puct_args(e, q, a);
    if (st != SN_OK) return st;
    if (r0 < 0 || nr < 1 || !ro_out) return set_error(SN_EINVAL, "need r0 >= 0, nr >= 1 and an output buffer");
    hipStream_t s = (hipStream_t)stream;
    const int64_t lanes = a.D * nr;
    SN_DISPATCH_N(e->s.N, hipLaunchKernelGGL((k_puct_deal_batch<NN>), dim3(grid_for(lanes)), dim3(kBlock), 0, s, e->s, a,
                                             (uint32_t)r0, nr, (int32_t*)ro_out));
    HIP_TRY(hipGetLastError());
    return SN_OK;
}

sn_status sn_puct_rows(sn_env* e, const sn_puct* q, int n_cur, void* rows, int bf16, void* stream) {
    PuctArgs a{};
    sn_status st = puct_args(e, q, a);
    if (st != SN_OK) return st;
    if (n_cur < 1 || n_cur > a.n) return set_error(SN_EINVAL, "n_cur out of range");
    const int64_t total = a.D * e->s.N * n_cur;
    hipStream_t s = (hipStream_t)stream;
    if (bf16)
        hipLaunchKernelGGL(k_puct_rows<__hip_bfloat16>, dim3(grid_for(total)), dim3(kBlock), 0, s, a, e->s.N, n_cur,
                           (__hip_bfloat16*)rows);
    else
        hipLaunchKernelGGL(k_puct_rows<float>, dim3(grid_for(total)), dim3(kBlock), 0, s, a, e->s.N, n_cur, (float*)rows);
    HIP_TRY(hipGetLastError());
    return SN_OK;
}

sn_status sn_puct_step(sn_env* e, const sn_puct* q, const float* logits, int t, int n_cur, void* stream) {
    PuctArgs a{};
    sn_status st = puct_args(e, q, a);
    if (st != SN_OK) return st;
    if (n_cur < 1 || n_cur > a.n || t < 0 || t + n_cur != a.n) return set_error(SN_EINVAL, "t / n_cur inconsistent");
    hipStream_t s = (hipStream_t)stream;
    const int ls = q->logit_stride > 1 ? q->logit_stride : 1;
    const char* sv = getenv("SECHS_PUCT_STEP_SEATS");  // "0": the one-lane-per-decision kernel (A/B, tests)
    const int seat_lanes = (sv && sv[0] == '0') ? 0 : 1;
    if (seat_lanes && e->s.N <= 8) {  // one lane per seat (k_puct_step_seats)
        const int Lw = e->s.N <= 2 ? 2 : e->s.N <= 4 ? 4 : 8;
        const int64_t lanes = a.D * Lw;
#define SN_STEP_SEATS(NN_, L_)                                                                                   \
    do {                                                                                                        \
        if (q->logit_bf16)                                                                                      \
            hipLaunchKernelGGL((k_puct_step_seats<NN_, L_, true>), dim3(grid_for(lanes)), dim3(kBlock), 0, s,  \
                               e->s, a, (const void*)logits, ls, t, n_cur);                                     \
        else                                                                                                    \
            hipLaunchKernelGGL((k_puct_step_seats<NN_, L_, false>), dim3(grid_for(lanes)), dim3(kBlock), 0, s, \
                               e->s, a, (const void*)logits, ls, t, n_cur);                                     \
    } while (0)
        switch (e->s.N) {
            case 1: SN_STEP_SEATS(1, 2); break;
            case 2: SN_STEP_SEATS(2, 2); break;
            case 3: SN_STEP_SEATS(3, 4); break;
            case 4: SN_STEP_SEATS(4, 4); break;
            case 5: SN_STEP_SEATS(5, 8); break;
            case 6: SN_STEP_SEATS(6, 8); break;
            case 7: SN_STEP_SEATS(7, 8); break;
            default: SN_STEP_SEATS(8, 8); break;
        }
#undef SN_STEP_SEATS
        HIP_TRY(hipGetLastError());
        return SN_OK;
    }
    if (q->logit_bf16) {

        SN_DISPATCH_N(e->s.N, hipLaunchKernelGGL((k_puct_step<NN, true>), dim3(grid_for(a.D)), dim3(kBlock), 0, s, e->s, a,
                                                 (const void*)logits, ls, t, n_cur));
    } else {
        SN_DISPATCH_N(e->s.N, hipLaunchKernelGGL((k_puct_step<NN, false>), dim3(grid_for(a.D)), dim3(kBlock), 0, s, e->s, a,
                                                 (const void*)logits, ls, t, n_cur));
    }
    HIP_TRY(hipGetLastError());
    return SN_OK;
}

sn_status sn_puct_mlp_seats(sn_env* e, const sn_puct* q, int n_cur, const void* w1s, const float* w1c, const void* w2,
                            const float* head, float* logits, void* stream) {
    PuctArgs a{};
    sn_status st = puct_args(e, q, a);
    if (st != SN_OK) return st;
    if (n_cur < 1 || n_cur > a.n) return set_error(SN_EINVAL, "n_cur out of range");
    if (!w1s || !w1c || !w2 || !head || !logits) return set_error(SN_EINVAL, "NULL argument");
    if ((((uintptr_t)w1s) | ((uintptr_t)w2) | ((uintptr_t)w1c) | ((uintptr_t)head)) & 15)
        return set_error(SN_EINVAL, "w1s / w2 / w1c / head must be 16-B aligned");
    const int64_t S = a.D * e->s.N;
    if (S * n_cur >= (1ll << 31)) return set_error(SN_EINVAL, "too many rows");
    const int cus = e->cus;  // persistent grid: two workgroups per CU (the kernel's occupancy) of the handle's device
    const int64_t groups = (S + kSeatBlock - 1) / kSeatBlock;
    hipLaunchKernelGGL(k_puct_mlp_seats, dim3((unsigned)std::min<int64_t>(groups, 2ll * cus)), dim3(kBlock), 0,
                       (hipStream_t)stream, a, e->s.N, n_cur, (const uint16_t*)w1s, w1c, (const uint16_t*)w2, head,
                       logits);
    HIP_TRY(hipGetLastError());
    return SN_OK;
}

sn_status sn_puct_rollouts(sn_env* e, const sn_puct* q, int r0, int nr, void* ro_base, const void* w1s, const float* w1c,
                           const void* w2, const float* head, void* stream) {
    PuctArgs a{};
    sn_status st = puct_args(e, q, a);
    if (st != SN_OK) return st;
    if (r0 < 0 || nr < 1 || !ro_base) return set_error(SN_EINVAL, "need r0 >= 0, nr >= 1 and the dealt states");
    if (!w1s || !w1c || !w2 || !head) return set_error(SN_EINVAL, "NULL argument");
    if ((((uintptr_t)w1s) | ((uintptr_t)w2) | ((uintptr_t)w1c) | ((uintptr_t)head)) & 15)
        return set_error(SN_EINVAL, "w1s / w2 / w1c / head must be 16-B aligned");
    if (e->s.N < 3 || e->s.N > 8) return set_error(SN_EUNSUPPORTED, "sn_puct_rollouts: 3 <= N <= 8");
    hipStream_t s = (hipStream_t)stream;
    const int Lw = e->s.N <= 2 ? 2 : e->s.N <= 4 ? 4 : 8;
    // decisions per wave's group: a wave carries its groups one after the other, so the launch
    // takes ceil(groups / waves) group-times; with the fewest rounds fixed, the smallest group
    // that keeps them (fewer seat rows and candidate tiles per group-step: a tournament's
    // decision count is rarely a multiple of 8 x the grid's waves)
    const int dg_max = kRollSeats / Lw;
    const int64_t slots = 8ll * e->cus;  // one 8-wave workgroup per CU
    const int64_t rounds = std::max<int64_t>(1, (a.D + dg_max * slots - 1) / (dg_max * slots));
    const int dg = (int)std::min<int64_t>(dg_max, std::max<int64_t>(1, (a.D + rounds * slots - 1) / (rounds * slots)));
    const int64_t groups = (a.D + dg - 1) / dg;
    const dim3 grid((unsigned)std::min<int64_t>((groups + 7) / 8, (int64_t)e->cus));
#define SN_ROLLOUTS(NN_, L_)                                                                                  \
    hipLaunchKernelGGL((k_puct_rollouts<NN_, L_>), grid, dim3(512), 0, s, e->s, a, r0, nr, (int32_t*)ro_base, \
                       (const uint16_t*)w1s, w1c, (const uint16_t*)w2, head, dg)
    switch (e->s.N) {
        case 3: SN_ROLLOUTS(3, 4); break;
        case 4: SN_ROLLOUTS(4, 4); break;
        case 5: SN_ROLLOUTS(5, 8); break;
        case 6: SN_ROLLOUTS(6, 8); break;
        case 7: SN_ROLLOUTS(7, 8); break;
        default: SN_ROLLOUTS(8, 8); break;
    }
#undef SN_ROLLOUTS
    HIP_TRY(hipGetLastError());
    return SN_OK;
}

sn_status sn_debug_puct_phases(uint64_t* out, int n) {
    if (!out || n < 1) return set_error(SN_EINVAL, "NULL argument");
#ifdef SECHS_PHASE_PROF
    unsigned long long h[8];
    HIP_TRY(hipDeviceSynchronize());
    HIP_TRY(hipMemcpyFromSymbol(h, HIP_SYMBOL(g_puct_phase), sizeof(h)));
    for (int k = 0; k < n; k++) out[k] = (k < 8) ? (uint64_t)h[k] : 0ull;
    const unsigned long long z[8] = {};
    HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(g_puct_phase), z, sizeof(z)));
    return SN_OK;
#else
    return set_error(SN_EUNSUPPORTED, "phase counters: build libsechs_prof.so (-DSECHS_PHASE_PROF)");
#endif
}

sn_status sn_puct_choose(sn_env* e, const sn_puct* q, int32_t* actions, int32_t* best_index, void* stream) {
    PuctArgs a{};
    sn_status st = puct_args(e, q, a);
    if (st != SN_OK) return st;
    hipLaunchKernelGGL(k_puct_choose, dim3(grid_for(a.D)), dim3(kBlock), 0, (hipStream_t)stream, e->s, a, actions,
                       best_index);
    HIP_TRY(hipGetLastError());
    return SN_OK;
}

sn_status sn_pcv_choose(sn_env* e, const sn_puct* q, const float* heads, int32_t* actions, int32_t* best_index,
                        float* log_prob, float* value, void* stream) {
    if (!heads || !actions) return set_error(SN_EINVAL, "NULL argument");
    PuctArgs a{};
    sn_status st = puct_args(e, q, a);
    if (st != SN_OK) return st;
    if (a.n < 1) return set_error(SN_EINVAL, "hand size must be >= 1");
    hipLaunchKernelGGL(k_pcv_choose, dim3(grid_for(a.D)), dim3(kBlock), 0, (hipStream_t)stream, e->s, a, heads,
                       actions, best_index, log_prob, value);
    HIP_TRY(hipGetLastError());
    return SN_OK;
}

sn_status sn_policy_sample(sn_env* e, const sn_puct* q, const float* logits, int32_t* actions, int32_t* index,
                           float* log_prob, float* entropy, void* stream) {
    if (!logits || !actions) return set_error(SN_EINVAL, "NULL argument");
    PuctArgs a{};
    sn_status st = puct_args(e, q, a);
    if (st != SN_OK) return st;
    hipLaunchKernelGGL(k_policy_sample, dim3(grid_for(a.D)), dim3(kBlock), 0, (hipStream_t)stream, e->s, a, logits,
                       actions, index, log_prob, entropy);
    HIP_TRY(hipGetLastError());
    return SN_OK;
}

sn_status sn_puct_score(int64_t D, const int32_t* n, const int32_t* stats, const int32_t* hist, const float* probs,
                        double c_puct, double* pucts, int32_t* choice, void* stream) {
    if (D <= 0 || !n || !stats || !hist || !probs || !pucts || !choice) return set_error(SN_EINVAL, "bad argument");
    hipLaunchKernelGGL(k_puct_score, dim3(grid_for(D)), dim3(kBlock), 0, (hipStream_t)stream, D, kHand, n, stats, hist,
                       probs, c_puct, pucts, choice);
    HIP_TRY(hipGetLastError());
    return SN_OK;
}

}  // extern "C"

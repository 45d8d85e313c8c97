// sechs_mcs.hip -- Monte-Carlo search (MCSAgent, agents/mcts.py:17-188) on gfx950.
//
// Two engines:
//  * stratified (BASELINE config 3): for every (game, seat) decision, R
//    playouts per legal first move, one lane per playout, one workgroup per
//    (decision, move).  Opponent hands are dealt from the seat's card memory
//    and all moves after the first are uniform, as in the reference's
//    _draw_env/_play_out (mcts.py:108-154); the sums are reduced in-block and
//    the move with the best mean wins (mcts.py:156-165).  Random words come
//    from Philox keyed (seed ^ decision step, seat/move/playout, game id).
//  * reference-exact: one lane runs a whole MCSAgent.forward (n_mc
//    sequential playouts) on a numpy MT19937 stream, reproducing the
//    reference's global-RNG order draw for draw.  Used by the drop-in
//    MCSAgent (numpy global state bridged in and out) and by a whole-game
//    kernel that replays GameSession(MCSAgent / DrunkHamster seats).
#include "sechs_mcs.h"
#include "sechs_mcs_wave.h"

using namespace sechs;

// ============================================================================
// stratified engine
// ============================================================================
// avail layout: [4][B*N] u32 (word-major, decision = g*N + p)
__global__ void k_mcs_memorize(DevState s, uint32_t* avail, int mcs_cards) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t D = s.B * s.N;
    if (i >= D) return;
    const int64_t g = i / s.N;
    const int p = (int)(i - g * s.N);
    const Hand h = load_hand(s, p, g);
    u32x4 m = {avail[i], avail[D + i], avail[2 * D + i], avail[3 * D + i]};
    m = memorize(m, hand_len(h), (uint32_t)mcs_cards, h, load_board(s, g));
    avail[i] = m.x, avail[D + i] = m.y, avail[2 * D + i] = m.z, avail[3 * D + i] = m.w;
}

struct McsArgs {
    const uint32_t* avail;  // [4][B*N]
    int32_t* sums;          // [B*N][10]
    int32_t* playouts;      // optional [B*N][10][R]: every playout's return
    uint32_t seed_lo, seed_hi, step, rollouts;
};

// one playout (mcts.py:108-154) from decision (g, p) with first move legal[a]
template <int N>
__device__ __forceinline__ int32_t playout(PhiloxGen& gen, ByteBuf& buf, const Board& root, const Hand& me, uint32_t n,
                                           u32x4 av, uint32_t a) {
    Game<N> R;
    R.hand[0] = me;
    R.b = root;
    uint32_t left = set_count(av);
    // _deal_hands: opponents' hands drawn without replacement from the memory
#pragma unroll
    for (int q = 1; q < N; q++) {
        u32x4 set = {0u, 0u, 0u, 0u};
        for (uint32_t i = 0; i < n && left > 0u; i++) {
            const uint32_t k = rng_interval(gen, buf, left - 1u);
            const uint32_t c = set_select(av, k);
            av = clear_bit(av, c);
            set = set_bit(set, c);
            left--;
        }
        R.hand[q] = hand_from_set(set);
    }
    int32_t outcome = 0;
    for (uint32_t t = 0; t < n; t++) {
        const uint32_t cur = n - t;
        uint32_t card[N], pen[N];
#pragma unroll
        for (int q = 0; q < N; q++) {
            const uint32_t idx = (q == 0 && t == 0) ? a : rng_interval(gen, buf, cur - 1u);
            card[q] = hand_get(R.hand[q], idx);
            hand_del(R.hand[q], idx);
        }
        resolve<N>(R.b, card, pen);
        outcome -= (int32_t)pen[0];
    }
    return outcome;
}

// grid (B*N, 10, R / blockDim), block = min(R, 256) playouts; the block
// sums land in sums[dec][move] by integer atomics (order-independent)
template <int N>
__global__ __launch_bounds__(kBlock) void k_mcs_rollouts(DevState s, McsArgs a) {
    __shared__ int32_t part[kBlock / 64];
    const int64_t dec = blockIdx.x;
    const uint32_t act = blockIdx.y;
    const int64_t g = dec / N;
    const int p = (int)(dec - g * N);
    const Hand me = load_hand(s, p, g);
    const uint32_t n = hand_len(me);
    if (act >= n || n <= 1u) return;  // uniform per block
    const int64_t D = s.B * N;
    const u32x4 av = {a.avail[dec], a.avail[D + dec], a.avail[2 * D + dec], a.avail[3 * D + dec]};
    const Board root = load_board(s, g);
    PhiloxGen gen;
    ByteBuf buf;
    const uint64_t gid = s.game_offset + (uint64_t)g;
    const uint32_t r = blockIdx.z * blockDim.x + threadIdx.x;  // playout index
    const uint64_t stream = ((uint64_t)(uint32_t)gid << 32) | ((uint64_t)p << 24) | ((uint64_t)act << 16) | r;
    gen.load(a.seed_lo ^ a.step, a.seed_hi, stream, 0ull, buf);
    int32_t v = playout<N>(gen, buf, root, me, n, av, act);
    if (a.playouts) a.playouts[(dec * kHand + act) * a.rollouts + r] = v;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    if ((threadIdx.x & 63u) == 0u) part[threadIdx.x >> 6] = v;
    __syncthreads();
    if (threadIdx.x == 0) {
        int32_t tot = 0;
        for (uint32_t w = 0; w < (blockDim.x >> 6); w++) tot += part[w];
        atomicAdd(&a.sums[dec * kHand + act], tot);
    }
}

// _choose_action_from_outcomes with equal playout counts: argmax of the
// sums in legal order, strict '>' so ties keep the lowest card (mcts.py:156-165)
__global__ void k_mcs_choose(DevState s, const int32_t* sums, int32_t* actions) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= s.B * s.N) return;
    const int64_t g = i / s.N;
    const int p = (int)(i - g * s.N);
    const Hand h = load_hand(s, p, g);
    const uint32_t n = hand_len(h);
    int32_t act = -1;
    if (n == 1u) {
        act = (int32_t)hand_get(h, 0u);
    } else if (n > 1u) {
        uint32_t best = 0;
        int32_t bs = sums[i * kHand];
        for (uint32_t k = 1; k < n; k++) {
            const int32_t v = sums[i * kHand + k];
            if (v > bs) bs = v, best = k;
        }
        act = (int32_t)hand_get(h, best);
    }
    actions[i] = act;
}

// ============================================================================
// reference-exact engine (numpy MT19937 streams): mcs_decide_exact, sechs_mcs.h
// ============================================================================
// whole GameSession games with MCSAgent seats (bit p of mcs_seats) and
// DrunkHamster seats, one lane per game, on the env's numpy streams:
// reset + 10 steps, exactly the reference's global-RNG call order
struct ExactArgs {
    uint32_t mcs_seats, mcs_cards;
    int mc_per_card, mc_max;
    int32_t* actions;  // [10][B][N]
    int32_t* rewards;  // [10][B][N]
    int32_t* status;   // [B]: 0 ok, 1 = the reference would have raised (Q6)
};

template <int N>
__global__ __launch_bounds__(kBlock) void k_mcs_play_exact(DevState s, ExactArgs a) {
    __shared__ uint8_t lds[kBlock * kDeckStride];
    const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= s.B) return;
    uint8_t* mine = lds + threadIdx.x * kDeckStride;
    MtGen gen;
    ByteBuf buf;
    RngOf<RNG_NUMPY_MT>::load(s, g, gen, buf);
    Game<N> G;
    deal_shuffle<N>(gen, buf, mine, s.C, G);
    u32x4 mem[N];
#pragma unroll
    for (int p = 0; p < N; p++) mem[p] = u32x4{0u, 0u, 0u, 0u};
    int32_t status = 0;
    for (int t = 0; G.n > 0u; t++) {
        uint32_t card[N], idx[N], pen[N];
#pragma unroll
        for (int p = 0; p < N; p++) {
            if ((a.mcs_seats >> p) & 1u) {
                mem[p] = memorize(mem[p], G.n, a.mcs_cards, G.hand[p], G.b);
                if (G.n == 1u) {
                    idx[p] = 0u;
                } else {
                    int32_t sum[kHand], cnt[kHand];
                    bool q6 = false;
                    const uint32_t c = mcs_decide_exact<N>(gen, buf, mine, G.b, G.hand[p], G.n, mem[p], a.mc_per_card,
                                                           a.mc_max, sum, cnt, &q6);
                    if (q6) status = 1;
                    idx[p] = (uint32_t)hand_find(G.hand[p], c);
                }
            } else {
                idx[p] = rng_interval(gen, buf, G.n - 1u);
            }
            card[p] = hand_get(G.hand[p], idx[p]);
        }
#pragma unroll
        for (int p = 0; p < N; p++) hand_del(G.hand[p], idx[p]);
        resolve<N>(G.b, card, pen);
        G.n -= 1u;
#pragma unroll
        for (int p = 0; p < N; p++) {
            G.score[p] += (int32_t)pen[p];
            if (a.actions) a.actions[((int64_t)t * s.B + g) * N + p] = (int32_t)card[p];
            if (a.rewards) a.rewards[((int64_t)t * s.B + g) * N + p] = -(int32_t)pen[p];
        }
    }
    if (a.status) a.status[g] = status;
    store_game<N>(s, g, G);
    RngOf<RNG_NUMPY_MT>::store(s, g, gen, buf);
}

struct DecideArgs {
    int64_t D;
    const int8_t* board;    // [D][4][6]
    const int8_t* hand;     // [D][10]
    const uint32_t* avail;  // [D][4]
    int mc_per_card, mc_max;
    uint32_t* mt_keys;      // [D][624] numpy form, in/out
    int32_t* mt_pos;        // [D] numpy pos, in/out
    int32_t* actions;       // [D]
    int32_t* sums;          // [D][10]
    int32_t* counts;        // [D][10]
};

// MCSAgent decisions (sn_mcs_decide_exact), one wave each (sechs_mcs_wave.h):
// the numpy key and pos in LDS, the playouts' draws decoded 64 words per instruction and
// played 64 at a time in the lanes; same words, same order, same outputs.
template <int N>
__global__ __launch_bounds__(64) void k_mcs_decide_wave(DecideArgs a) {
    __shared__ WmcsLds L;
    __shared__ uint32_t head[64];
    const int64_t d = blockIdx.x;
    const uint32_t lane = threadIdx.x;
    uint32_t* key = a.mt_keys + d * kMtN;
    WaveMt m{L.st, L.stage, 0u, 0u, 0u, 0u, false, head};
    wmt_load(m, key, mt_code_from_numpy(a.mt_pos[d]), lane);
    u32x4 hs = {0u, 0u, 0u, 0u};
    for (int k = 0; k < kHand; k++) {
        const int c = a.hand[d * kHand + k];
        if (c >= 0) hs = set_bit(hs, (uint32_t)c);
    }
    const Hand me = hand_from_set(hs);
    uint32_t lo[4], hi[4];
#pragma unroll
    for (int r = 0; r < kRows; r++) {
        uint32_t l = 0, card4 = 0, len = 0, heads = 0, end = 0;
        for (int i = 0; i < kThreshold; i++) {
            const int c = a.board[(d * kRows + r) * kThreshold + i];
            if (c < 0) continue;
            if (len < 4) l |= (uint32_t)c << (8 * len);
            else card4 = (uint32_t)c;
            heads += heads_of((uint32_t)c);
            end = (uint32_t)c;
            len++;
        }
        lo[r] = l, hi[r] = (card4 & 0xFFu) | (len << 8) | (heads << 16) | (end << 24);
    }
    Board b;
    b.lo = u32x4{lo[0], lo[1], lo[2], lo[3]};
    b.hi = u32x4{hi[0], hi[1], hi[2], hi[3]};
    const u32x4 av = {a.avail[d * 4 + 0], a.avail[d * 4 + 1], a.avail[d * 4 + 2], a.avail[d * 4 + 3]};
    const uint32_t n = hand_len(me);
    bool q6 = false;
    uint32_t c = hand_get(me, 0u);
    int32_t* sums = a.sums ? a.sums + d * kHand : nullptr;
    int32_t* counts = a.counts ? a.counts + d * kHand : nullptr;
    if (n > 1u) {
        c = wmcs_decide<N>(m, L, b, me, n, av, a.mc_per_card, a.mc_max, &q6, lane, sums, counts);
    } else if (lane < (uint32_t)kHand) {
        if (sums) sums[lane] = 0;
        if (counts) counts[lane] = 0;
    }
    const int32_t pos = wmt_store_numpy(m, key, lane);
    if (lane == 0u) {
        a.actions[d] = q6 ? -(int32_t)c - 2 : (int32_t)c;  // -(card)-2 flags quirk Q6
        a.mt_pos[d] = pos;
    }
}

// ============================================================================
// C ABI
// ============================================================================
extern "C" {

sn_status sn_mcs_memorize(sn_env* e, uint32_t* avail, int mcs_num_cards, void* stream) {
    if (!e || !avail) return set_error(SN_EINVAL, "NULL argument");
    if (mcs_num_cards < 1 || mcs_num_cards > 128) return set_error(SN_EINVAL, "mcs_num_cards must be in 1..128");
    hipLaunchKernelGGL(k_mcs_memorize, dim3(grid_for(e->s.B * e->s.N)), dim3(kBlock), 0, (hipStream_t)stream, e->s,
                       avail, mcs_num_cards);
    HIP_TRY(hipGetLastError());
    return SN_OK;
}

sn_status sn_mcs_rollouts_ex(sn_env* e, const uint32_t* avail, int rollouts, uint64_t seed, uint32_t decision_step,
                             int32_t* sums, int32_t* playouts, void* stream) {
    if (!e || !avail || !sums) return set_error(SN_EINVAL, "NULL argument");
    if (rollouts < 64 || rollouts > 65536 || (rollouts & 63) || (rollouts > kBlock && rollouts % kBlock))
        return set_error(SN_EINVAL, "rollouts must be 64, 128, 192 or a multiple of 256 (<= 65536)");
    const DevState& s = e->s;
    if (s.B * s.N > 0x7FFFFFFF) return set_error(SN_EINVAL, "too many decisions for one launch");
    McsArgs a{};
    a.avail = avail;
    a.sums = sums;
    a.playouts = playouts;
    a.rollouts = (uint32_t)rollouts;
    a.seed_lo = (uint32_t)seed, a.seed_hi = (uint32_t)(seed >> 32), a.step = decision_step;
    const unsigned block = rollouts < kBlock ? (unsigned)rollouts : (unsigned)kBlock;
    const dim3 grid((unsigned)(s.B * s.N), kHand, (unsigned)rollouts / block);
    hipStream_t st = (hipStream_t)stream;
    HIP_TRY(hipMemsetAsync(sums, 0, sizeof(int32_t) * kHand * s.B * s.N, st));
    SN_DISPATCH_N(s.N, hipLaunchKernelGGL((k_mcs_rollouts<NN>), grid, dim3(block), 0, st, s, a));
    HIP_TRY(hipGetLastError());
    return SN_OK;
}

sn_status sn_mcs_rollouts(sn_env* e, const uint32_t* avail, int rollouts, uint64_t seed, uint32_t decision_step,
                          int32_t* sums, void* stream) {
    return sn_mcs_rollouts_ex(e, avail, rollouts, seed, decision_step, sums, nullptr, stream);
}

sn_status sn_mcs_choose(sn_env* e, const int32_t* sums, int32_t* actions, void* stream) {
    if (!e || !sums || !actions) return set_error(SN_EINVAL, "NULL argument");
    hipLaunchKernelGGL(k_mcs_choose, dim3(grid_for(e->s.B * e->s.N)), dim3(kBlock), 0, (hipStream_t)stream, e->s, sums,
                       actions);
    HIP_TRY(hipGetLastError());
    return SN_OK;
}

sn_status sn_mcs_play_exact(sn_env* e, uint32_t mcs_seats, int mc_per_card, int mc_max, int32_t* actions,
                            int32_t* rewards, int32_t* status, void* stream) {
    if (!e) return set_error(SN_EINVAL, "NULL argument");
    if (e->s.rng_mode != SN_RNG_NUMPY_MT) return set_error(SN_EINVAL, "reference-exact MCS needs the numpy-MT RNG mode");
    if (sn_pipe_sync(e, (hipStream_t)stream) != SN_OK) return SN_EHIP;
    if (mc_per_card < 0 || mc_max < 0) return set_error(SN_EINVAL, "mc_per_card and mc_max must be >= 0");
    e->phase = -1;
    ExactArgs a{};
    a.mcs_seats = mcs_seats, a.mcs_cards = kMaxCards, a.mc_per_card = mc_per_card, a.mc_max = mc_max;
    a.actions = actions, a.rewards = rewards, a.status = status;
    const DevState& s = e->s;
    hipStream_t st = (hipStream_t)stream;
    SN_DISPATCH_N(s.N, hipLaunchKernelGGL((k_mcs_play_exact<NN>), dim3(grid_for(s.B)), dim3(kBlock), 0, st, s, a));
    HIP_TRY(hipGetLastError());
    return SN_OK;
}

sn_status sn_mcs_decide_exact(int device, int64_t D, int num_players, const int8_t* board, const int8_t* hand,
                              const uint32_t* avail, int mc_per_card, int mc_max, uint32_t* mt_keys, int32_t* mt_pos,
                              int32_t* actions, int32_t* sums, int32_t* counts, void* stream) {
    if (D <= 0 || D > 0x7FFFFFFF || !board || !hand || !avail || !mt_keys || !mt_pos || !actions)
        return set_error(SN_EINVAL, "bad argument");
    if (mc_per_card < 0 || mc_max < 0) return set_error(SN_EINVAL, "mc_per_card and mc_max must be >= 0");
    HIP_TRY(hipSetDevice(device));
    DecideArgs a{};
    a.D = D, a.board = board, a.hand = hand, a.avail = avail, a.mc_per_card = mc_per_card, a.mc_max = mc_max;
    a.mt_keys = mt_keys, a.mt_pos = mt_pos, a.actions = actions, a.sums = sums, a.counts = counts;
    hipStream_t st = (hipStream_t)stream;
    SN_DISPATCH_N(num_players, hipLaunchKernelGGL((k_mcs_decide_wave<NN>), dim3((unsigned)D), dim3(64), 0, st, a));
    HIP_TRY(hipGetLastError());
    return SN_OK;
}

}  // extern "C"

// sechs_env.hip -- vectorised SechsNimmtEnv for gfx950 + the C ABI (include/sechs.h).
//
// Device state is struct-of-arrays over games (lane g reads element g of
// every array, so each load/store instruction of a wave is one contiguous
// 256-B segment):
//   hand   [N][4][B] u32   128-bit card set per seat
//   row_lo [4][B]    u32   cards 0..3 of each row
//   row_hi [4][B]    u32   card4 | len<<8 | heads<<16 | end<<24
//   score  [N][B]    i32   penalties this episode (env.py:32)
//   sum_res[N][B]    i32   sum of finished episodes' results (-penalty)
//   episodes [B]     i32
//   mt [B][624] u32 + mt_pos [B]   (numpy-compat mode; per-game AoS so a
//                                   lane's lazy twist walks its own lines)
//   ctr [B] u64                    (philox mode: words consumed)
// A launch loads a game into VGPRs, plays `steps` env-steps and stores it
// back; the only per-step HBM traffic is the caller's outputs and, in
// numpy-compat mode, the MT19937 words.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>
#include <new>
#include <string>

#include "../../include/sechs.h"
#include "sechs_device.h"

using namespace sechs;

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
};

struct sn_env {
    int device;
    DevState s;
};

constexpr int kBlock = 256;
constexpr int kDeckStride = 108;  // 27 dwords: odd stride -> conflict-free LDS lanes

// ---------------------------------------------------------------- rng glue
template <int MODE>
struct RngOf;
template <>
struct RngOf<RNG_NUMPY_MT> {
    using T = MtRng;
    static __device__ __forceinline__ T load(const DevState& s, int64_t g) {
        T r;
        r.st = s.mt + g * kMtN;
        r.pos = s.mt_pos[g];
        return r;
    }
    static __device__ __forceinline__ void store(const DevState& s, int64_t g, const T& r) { s.mt_pos[g] = r.pos; }
};
template <>
struct RngOf<RNG_PHILOX> {
    using T = PhiloxRng;
    static __device__ __forceinline__ T load(const DevState& s, int64_t g) {
        T r;
        r.k0 = (uint32_t)s.seed;
        r.k1 = (uint32_t)(s.seed >> 32);
        uint64_t gid = s.game_offset + (uint64_t)g;
        r.s0 = (uint32_t)gid;
        r.s1 = (uint32_t)(gid >> 32);
        r.ctr = s.ctr[g];
        if (r.ctr & 3u) r.refill();
        else r.buf[0] = r.buf[1] = r.buf[2] = r.buf[3] = 0u;
        return r;
    }
    static __device__ __forceinline__ void store(const DevState& s, int64_t g, const T& r) { s.ctr[g] = r.ctr; }
};

// ---------------------------------------------------------------- game in VGPRs
template <int N>
struct Game {
    Hand hand[N];
    Board b;
    int32_t score[N];
};

template <int N>
__device__ __forceinline__ void load_game(const DevState& s, int64_t g, Game<N>& G) {
    const int64_t B = s.B;
#pragma unroll
    for (int p = 0; p < N; p++) {
#pragma unroll
        for (int w = 0; w < 4; w++) G.hand[p].w[w] = s.hand[(int64_t)(p * 4 + w) * B + g];
        G.score[p] = s.score[(int64_t)p * B + g];
    }
#pragma unroll
    for (int r = 0; r < kRows; r++) {
        G.b.lo[r] = s.row_lo[(int64_t)r * B + g];
        G.b.hi[r] = s.row_hi[(int64_t)r * B + g];
    }
}

template <int N>
__device__ __forceinline__ void store_game(const DevState& s, int64_t g, const Game<N>& G) {
    const int64_t B = s.B;
#pragma unroll
    for (int p = 0; p < N; p++) {
#pragma unroll
        for (int w = 0; w < 4; w++) s.hand[(int64_t)(p * 4 + w) * B + g] = G.hand[p].w[w];
        s.score[(int64_t)p * B + g] = G.score[p];
    }
#pragma unroll
    for (int r = 0; r < kRows; r++) {
        s.row_lo[(int64_t)r * B + g] = G.b.lo[r];
        s.row_hi[(int64_t)r * B + g] = G.b.hi[r];
    }
}

// env.py:99-112 _deal after np.random.shuffle(arange(C)) (legacy
// Fisher-Yates from the end, j = random_interval(i)).  The deck lives in
// this lane's LDS slot; hands come from deck[0..10N), rows from deck[C-1-r].
template <int N, class R>
__device__ __forceinline__ void deal_shuffle(R& rng, uint8_t* deck, int C, Game<N>& G) {
    for (int i = 0; i < C; i += 4) *(uint32_t*)(deck + i) = (uint32_t)i * 0x01010101u + 0x03020100u;
    for (int i = C - 1; i >= 1; --i) {
        uint32_t j = rng_interval(rng, (uint32_t)i);
        uint8_t di = deck[i], dj = deck[j];
        deck[i] = dj;
        deck[j] = di;
    }
#pragma unroll
    for (int p = 0; p < N; p++) {
        hand_clear(G.hand[p]);
#pragma unroll
        for (int k = 0; k < kHand; k++) hand_add(G.hand[p], deck[kHand * p + k]);
        G.score[p] = 0;
    }
#pragma unroll
    for (int r = 0; r < kRows; r++) row_start(G.b, r, deck[C - 1 - r]);
}

template <int N>
__device__ __forceinline__ void deal_given(const uint8_t* deck, int C, Game<N>& G) {
#pragma unroll
    for (int p = 0; p < N; p++) {
        hand_clear(G.hand[p]);
#pragma unroll
        for (int k = 0; k < kHand; k++) hand_add(G.hand[p], deck[kHand * p + k]);
        G.score[p] = 0;
    }
#pragma unroll
    for (int r = 0; r < kRows; r++) row_start(G.b, r, deck[C - 1 - r]);
}

// ---------------------------------------------------------------- observation
// env.py:188-212 for one seat, as 12 little-endian u32 words (48 bytes,
// bytes >= L zero): [hand asc, -1 pad to 10][N][lens][ends][heads][4x6 board]
template <bool SUMM>
__device__ __forceinline__ void obs_words(Hand h, int N, const Board& b, uint32_t (&w)[12]) {
#pragma unroll
    for (int i = 0; i < 12; i++) w[i] = 0u;
    uint32_t n = hand_count(h);
#pragma unroll
    for (int k = 0; k < kHand; k++) {
        uint32_t c = ((uint32_t)k < n) ? hand_pop_min(h) : 0xFFu;
        w[k >> 2] |= (c & 0xFFu) << (8 * (k & 3));
    }
    int pos = 10;
    w[pos >> 2] |= ((uint32_t)N & 0xFFu) << (8 * (pos & 3));
    pos++;
    if (SUMM) {
#pragma unroll
        for (int r = 0; r < kRows; r++, pos++) w[pos >> 2] |= row_len(b, r) << (8 * (pos & 3));
#pragma unroll
        for (int r = 0; r < kRows; r++, pos++) w[pos >> 2] |= row_end(b, r) << (8 * (pos & 3));
#pragma unroll
        for (int r = 0; r < kRows; r++, pos++) w[pos >> 2] |= row_heads(b, r) << (8 * (pos & 3));
    }
#pragma unroll
    for (int r = 0; r < kRows; r++) {
        const uint32_t len = row_len(b, r);
#pragma unroll
        for (int i = 0; i < kThreshold; i++, pos++) {
            uint32_t c = ((uint32_t)i < len) ? row_card(b, r, i) : 0xFFu;
            w[pos >> 2] |= c << (8 * (pos & 3));
        }
    }
}

// store one seat's obs row of `stride` bytes (stride % 4 == 0, >= L; bytes
// past the 48 packed ones are zero).  16-B stores when the row allows it.
__device__ __forceinline__ void store_obs_row(int8_t* dst, const uint32_t (&w)[12], int stride) {
    if ((stride & 15) == 0 && (((uintptr_t)dst) & 15) == 0) {  // stride >= 48 here
        uint4* d = (uint4*)dst;
        d[0] = make_uint4(w[0], w[1], w[2], w[3]);
        d[1] = make_uint4(w[4], w[5], w[6], w[7]);
        d[2] = make_uint4(w[8], w[9], w[10], w[11]);
        for (int i = 3; i < (stride >> 4); i++) d[i] = make_uint4(0u, 0u, 0u, 0u);
    } else {
        uint32_t* d = (uint32_t*)dst;
        const int nw = stride >> 2;
#pragma unroll
        for (int i = 0; i < 12; i++)
            if (i < nw) d[i] = w[i];
        for (int i = 12; i < nw; i++) d[i] = 0u;
    }
}

// ============================================================================
// kernels
// ============================================================================
__global__ void k_seed(DevState s) {
    const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= s.B) return;
    if (s.rng_mode == RNG_NUMPY_MT) {
        // np.random.seed(seed + gid): init_genrand, numpy pos = 624 (== lazy 0)
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

template <int N, int MODE>
__global__ __launch_bounds__(kBlock) void k_reset(DevState s, const uint8_t* decks) {
    __shared__ uint8_t lds_deck[kBlock * kDeckStride];
    const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= s.B) return;
    Game<N> G;
    if (decks) {
        deal_given<N>(decks + g * s.C, s.C, G);
    } else {
        auto rng = RngOf<MODE>::load(s, g);
        deal_shuffle<N>(rng, lds_deck + threadIdx.x * kDeckStride, s.C, G);
        RngOf<MODE>::store(s, g, rng);
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
        hand_clear(G.hand[p]);
        for (int k = 0; k < kHand; k++) {
            int c = hands[(g * N + p) * kHand + k];
            if (c >= 0) hand_add(G.hand[p], (uint32_t)c);
        }
        G.score[p] = 0;
    }
#pragma unroll
    for (int r = 0; r < kRows; r++) {
        uint32_t lo = 0, hi = 0, len = 0, heads = 0, end = 0;
        for (int i = 0; i < kThreshold; i++) {
            int c = board[(g * kRows + r) * kThreshold + i];
            if (c < 0) continue;
            if (len < 4) lo |= (uint32_t)c << (8 * len);
            else hi = (uint32_t)c;
            heads += heads_of((uint32_t)c);
            end = (uint32_t)c;
            len++;
        }
        G.b.lo[r] = lo;
        G.b.hi[r] = (hi & 0xFFu) | (len << 8) | (heads << 16) | (end << 24);
    }
    store_game<N>(s, g, G);
}

struct PlayArgs {
    int steps, flags, obs_stride, pad_;
    const int32_t* actions;  // [B][N] (steps == 1) or NULL = DrunkHamster
    int32_t* rewards;        // [steps][B][N]
    uint8_t* done;           // [steps][B]
    uint8_t* actions_out;    // [steps][B][N]
    int8_t* obs;             // [steps][B][N][obs_stride]
    int32_t* invalid;        // [B]
};

template <int N, int MODE>
__global__ __launch_bounds__(kBlock) void k_play(DevState s, PlayArgs a) {
    __shared__ uint8_t lds_deck[kBlock * kDeckStride];
    const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= s.B) return;
    const int64_t B = s.B;
    Game<N> G;
    load_game<N>(s, g, G);
    auto rng = RngOf<MODE>::load(s, g);
    const bool summ = !(a.flags & SN_NO_SUMMARIES);
    for (int t = 0; t < a.steps; t++) {
        const uint32_t n = hand_count(G.hand[0]);
        if (a.obs) {
            int8_t* base = a.obs + ((int64_t)t * B + g) * N * a.obs_stride;
#pragma unroll
            for (int p = 0; p < N; p++) {
                uint32_t w[12];
                if (summ) obs_words<true>(G.hand[p], N, G.b, w);
                else obs_words<false>(G.hand[p], N, G.b, w);
                store_obs_row(base + p * a.obs_stride, w, a.obs_stride);
            }
        }
        uint32_t card[N], pen[N];
        int bad = -1;
        if (n == 0u) {
            bad = 0;  // finished game stepped without auto-reset: nothing to play
        } else if (a.actions) {
#pragma unroll
            for (int p = N - 1; p >= 0; p--) {
                int32_t c = a.actions[g * N + p];
                card[p] = (uint32_t)c;
                bool ok = c >= 0 && c < s.C && hand_has(G.hand[p], (uint32_t)c);
                bad = ok ? bad : p;
            }
        } else {
            // DrunkHamster for every seat, in seat order (play.py:38-41)
#pragma unroll
            for (int p = 0; p < N; p++) card[p] = hand_select(G.hand[p], rng_interval(rng, n - 1u));
        }
        if (a.invalid) a.invalid[g] = bad;
        if (bad >= 0) {
            if (a.rewards)
#pragma unroll
                for (int p = 0; p < N; p++) a.rewards[((int64_t)t * B + g) * N + p] = 0;
            if (a.done) a.done[(int64_t)t * B + g] = (n == 0u) ? 1 : 0;
            continue;
        }
#pragma unroll
        for (int p = 0; p < N; p++) hand_remove(G.hand[p], card[p]);
        resolve<N>(G.b, card, pen);
#pragma unroll
        for (int p = 0; p < N; p++) G.score[p] += (int32_t)pen[p];
        const bool done = (n == 1u);
        if (a.rewards)
#pragma unroll
            for (int p = 0; p < N; p++) a.rewards[((int64_t)t * B + g) * N + p] = -(int32_t)pen[p];
        if (a.actions_out)
#pragma unroll
            for (int p = 0; p < N; p++) a.actions_out[((int64_t)t * B + g) * N + p] = (uint8_t)card[p];
        if (a.done) a.done[(int64_t)t * B + g] = done ? 1 : 0;
        if (done && (a.flags & SN_AUTO_RESET)) {
#pragma unroll
            for (int p = 0; p < N; p++) s.sum_res[(int64_t)p * B + g] -= G.score[p];
            s.episodes[g] += 1;
            deal_shuffle<N>(rng, lds_deck + threadIdx.x * kDeckStride, s.C, G);
        }
    }
    store_game<N>(s, g, G);
    RngOf<MODE>::store(s, g, rng);
}

// obs in any dtype, one thread per (game, seat)
template <typename T>
__global__ void k_obs(DevState s, T* out, int stride, int summ) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= s.B * s.N) return;
    const int64_t g = i / s.N;
    const int p = (int)(i - g * s.N);
    Hand h;
#pragma unroll
    for (int w = 0; w < 4; w++) h.w[w] = s.hand[(int64_t)(p * 4 + w) * s.B + g];
    Board b;
#pragma unroll
    for (int r = 0; r < kRows; r++) {
        b.lo[r] = s.row_lo[(int64_t)r * s.B + g];
        b.hi[r] = s.row_hi[(int64_t)r * s.B + g];
    }
    uint32_t w[12];
    if (summ) obs_words<true>(h, s.N, b, w);
    else obs_words<false>(h, s.N, b, w);
    T* dst = out + i * stride;
    const int L = summ ? 47 : 35;
#pragma unroll
    for (int wi = 0; wi < 12; wi++)
#pragma unroll
        for (int bi = 0; bi < 4; bi++) {
            const int k = 4 * wi + bi;
            if (k < stride) dst[k] = (k < L) ? (T)(int8_t)((w[wi] >> (8 * bi)) & 0xFFu) : (T)0;
        }
    for (int k = 48; k < stride; k++) dst[k] = (T)0;
}

__global__ void k_hands(DevState s, int8_t* out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= s.B * s.N) return;
    const int64_t g = i / s.N;
    const int p = (int)(i - g * s.N);
    Hand h;
#pragma unroll
    for (int w = 0; w < 4; w++) h.w[w] = s.hand[(int64_t)(p * 4 + w) * s.B + g];
    uint32_t n = hand_count(h);
    for (int k = 0; k < kHand; k++) out[i * kHand + k] = ((uint32_t)k < n) ? (int8_t)hand_pop_min(h) : (int8_t)-1;
}

__global__ void k_board(DevState s, int8_t* out) {
    const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= s.B) return;
    Board b;
#pragma unroll
    for (int r = 0; r < kRows; r++) {
        b.lo[r] = s.row_lo[(int64_t)r * s.B + g];
        b.hi[r] = s.row_hi[(int64_t)r * s.B + g];
    }
#pragma unroll
    for (int r = 0; r < kRows; r++)
        for (int i = 0; i < kThreshold; i++)
            out[(g * kRows + r) * kThreshold + i] = ((uint32_t)i < row_len(b, r)) ? (int8_t)row_card(b, r, i) : (int8_t)-1;
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

static sn_status fail(sn_status st, const std::string& msg) {
    g_err = msg;
    return st;
}

#define HIP_TRY(expr)                                                                               \
    do {                                                                                            \
        hipError_t e_ = (expr);                                                                     \
        if (e_ != hipSuccess) return fail(SN_EHIP, std::string(#expr ": ") + hipGetErrorString(e_)); \
    } while (0)

static inline unsigned grid_for(int64_t n) { return (unsigned)((n + kBlock - 1) / kBlock); }

// instantiate f<N, MODE> for N in 1..10
#define SN_DISPATCH_N(N_, BODY)                         \
    switch (N_) {                                       \
        case 1: { constexpr int NN = 1; BODY; } break;  \
        case 2: { constexpr int NN = 2; BODY; } break;  \
        case 3: { constexpr int NN = 3; BODY; } break;  \
        case 4: { constexpr int NN = 4; BODY; } break;  \
        case 5: { constexpr int NN = 5; BODY; } break;  \
        case 6: { constexpr int NN = 6; BODY; } break;  \
        case 7: { constexpr int NN = 7; BODY; } break;  \
        case 8: { constexpr int NN = 8; BODY; } break;  \
        case 9: { constexpr int NN = 9; BODY; } break;  \
        case 10: { constexpr int NN = 10; BODY; } break; \
        default: return fail(SN_EINVAL, "num_players out of range"); \
    }

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
    DevState& s = e->s;
    s.B = num_games, s.N = num_players, s.C = num_cards, s.rng_mode = rng_mode;
    s.seed = seed, s.game_offset = game_offset;
    const int64_t B = num_games, N = num_players;
    struct {
        void** p;
        size_t bytes;
    } allocs[] = {
        {(void**)&s.hand, sizeof(uint32_t) * N * 4 * B},   {(void**)&s.row_lo, sizeof(uint32_t) * kRows * B},
        {(void**)&s.row_hi, sizeof(uint32_t) * kRows * B}, {(void**)&s.score, sizeof(int32_t) * N * B},
        {(void**)&s.sum_res, sizeof(int32_t) * N * B},     {(void**)&s.episodes, sizeof(int32_t) * B},
        {(void**)&s.mt_pos, sizeof(uint32_t) * B},         {(void**)&s.ctr, sizeof(uint64_t) * B},
        {(void**)&s.mt, rng_mode == SN_RNG_NUMPY_MT ? sizeof(uint32_t) * kMtN * B : 4},
    };
    for (auto& a : allocs) {
        if (hipMalloc(a.p, a.bytes) != hipSuccess) {
            sn_destroy(e);
            return fail(SN_ENOMEM, "hipMalloc of device state failed");
        }
        (void)hipMemset(*a.p, 0, a.bytes);
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

sn_status sn_destroy(sn_env* e) {
    if (!e) return SN_OK;
    (void)hipSetDevice(e->device);
    DevState& s = e->s;
    void* ps[] = {s.hand, s.row_lo, s.row_hi, s.score, s.sum_res, s.episodes, s.mt_pos, s.ctr, s.mt};
    for (void* p : ps)
        if (p) (void)hipFree(p);
    delete e;
    return SN_OK;
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
    const DevState& s = e->s;
    if (s.rng_mode == SN_RNG_NUMPY_MT) {
        SN_DISPATCH_N(s.N, hipLaunchKernelGGL((k_reset<NN, RNG_NUMPY_MT>), dim3(grid_for(s.B)), dim3(kBlock), 0, st, s, decks));
    } else {
        SN_DISPATCH_N(s.N, hipLaunchKernelGGL((k_reset<NN, RNG_PHILOX>), dim3(grid_for(s.B)), dim3(kBlock), 0, st, s, decks));
    }
    HIP_TRY(hipGetLastError());
    return SN_OK;
}

sn_status sn_reset_to(sn_env* e, const int8_t* board, const int8_t* hands, void* stream) {
    if (!e || !board || !hands) return fail(SN_EINVAL, "NULL argument");
    hipStream_t st = (hipStream_t)stream;
    const DevState& s = e->s;
    SN_DISPATCH_N(s.N, hipLaunchKernelGGL((k_reset_to<NN>), dim3(grid_for(s.B)), dim3(kBlock), 0, st, s, board, hands));
    HIP_TRY(hipGetLastError());
    return SN_OK;
}

static sn_status launch_play(sn_env* e, const PlayArgs& a, hipStream_t st) {
    const DevState& s = e->s;
    if (s.rng_mode == SN_RNG_NUMPY_MT) {
        SN_DISPATCH_N(s.N, hipLaunchKernelGGL((k_play<NN, RNG_NUMPY_MT>), dim3(grid_for(s.B)), dim3(kBlock), 0, st, s, a));
    } else {
        SN_DISPATCH_N(s.N, hipLaunchKernelGGL((k_play<NN, RNG_PHILOX>), dim3(grid_for(s.B)), dim3(kBlock), 0, st, s, a));
    }
    HIP_TRY(hipGetLastError());
    return SN_OK;
}

sn_status sn_step(sn_env* e, const int32_t* actions, int32_t* rewards, uint8_t* done, int32_t* invalid, int flags,
                  void* stream) {
    if (!e) return fail(SN_EINVAL, "env is NULL");
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
    PlayArgs a{};
    a.steps = steps;
    a.flags = flags;
    a.obs_stride = obs_stride;
    a.rewards = rewards;
    a.done = done;
    a.actions_out = actions;
    a.obs = obs;
    return launch_play(e, a, (hipStream_t)stream);
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

sn_status sn_mt_get(sn_env* e, int64_t game, uint32_t* key, int32_t* pos) {
    if (!e || !key || !pos) return fail(SN_EINVAL, "NULL argument");
    if (e->s.rng_mode != SN_RNG_NUMPY_MT) return fail(SN_EINVAL, "env is not in numpy-compat RNG mode");
    if (game < 0 || game >= e->s.B) return fail(SN_EINVAL, "game out of range");
    HIP_TRY(hipSetDevice(e->device));
    HIP_TRY(hipDeviceSynchronize());
    uint32_t code = 0;
    HIP_TRY(hipMemcpy(key, e->s.mt + game * kMtN, sizeof(uint32_t) * kMtN, hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(&code, e->s.mt_pos + game, sizeof(uint32_t), hipMemcpyDeviceToHost));
    if (code >= (uint32_t)kMtN) {
        *pos = (int32_t)(code - kMtN);
    } else if (code == 0) {
        *pos = kMtN;
    } else {
        mt_finish_round(key, (int)code);
        *pos = (int32_t)code;
    }
    return SN_OK;
}

sn_status sn_mt_set(sn_env* e, int64_t game, const uint32_t* key, int32_t pos) {
    if (!e || !key) return fail(SN_EINVAL, "NULL argument");
    if (e->s.rng_mode != SN_RNG_NUMPY_MT) return fail(SN_EINVAL, "env is not in numpy-compat RNG mode");
    if (game < 0 || game >= e->s.B) return fail(SN_EINVAL, "game out of range");
    if (pos < 0 || pos > kMtN) return fail(SN_EINVAL, "pos must be in 0..624");
    HIP_TRY(hipSetDevice(e->device));
    HIP_TRY(hipDeviceSynchronize());
    uint32_t code = (pos == kMtN) ? 0u : (uint32_t)(kMtN + pos);
    HIP_TRY(hipMemcpy(e->s.mt + game * kMtN, key, sizeof(uint32_t) * kMtN, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(e->s.mt_pos + game, &code, sizeof(uint32_t), hipMemcpyHostToDevice));
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

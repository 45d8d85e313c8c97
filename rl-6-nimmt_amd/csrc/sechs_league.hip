// sechs_league.hip -- batched tournament with mixed agents on gfx950
// (Tournament.play_game, tournament.py:132-177, with the agents of run.py:20-40).
//
// A tournament handle (sn_league_config) plays one league game per slot at a
// time.  sn_league_rollout (sechs_env.hip) is the all-DrunkHamster fast path;
// sn_league_step here advances every slot's game by one env-step with any
// mix of agents, seats in seat order as GameSession.play_game calls them
// (play.py:38-41):
//   * DrunkHamster (agents/random.py:9): legal[random_interval(n-1)] on the
//     slot's numpy MT19937 stream;
//   * MCSAgent (agents/mcts.py:43-188): card memory + the reference-exact
//     search (sechs_mcs.h) on the same stream -- so a league of DrunkHamster
//     and MCSAgent seats replays the reference's seeded Tournament draw for
//     draw (golden F11 "dropin" leagues);
//   * external agents (the net agents: PUCTAgent, PUCTCustomedAgent,
//     BatchedACERAgent): their batched engines chose the card beforehand
//     (sechs_puct.hip over the handle's decision lists); it is checked
//     against the hand like env.py:114-118.
// A game that ends writes its record (seats word, results); the next game of
// every slot starts with sn_reset (the seat draw, then the deal: the next
// Tournament.play_game, tournament.py:132-138), so the roster may change
// between games (Tournament.evolve).
#include "sechs_mcs.h"
#include "sechs_mcs_wave.h"

using namespace sechs;

struct LeagueStepArgs {
    const int32_t* actions;  // [B][N] cards of external seats (may be NULL if no agent is external)
    int32_t* rewards;        // [B][N] (optional)
    int32_t* played;         // [B][N] cards played, -1 past k (optional)
    int32_t* records;        // [B][1 + N] per game that ended this step: seats word, results (optional)
    int32_t* invalid;        // [B] first seat whose external card is not in its hand, else -1 (optional)
    int32_t* status;         // [B] |= 1 where an MCSAgent move got no playout (quirk Q6; optional)
    uint64_t kinds;          // agent a's SN_AGENT_* in bits 4a..4a+3
    int32_t mpc[kLeagueMaxAgents], mmax[kLeagueMaxAgents];
};

// MCSAgent search for a game of k players (the agent's num_players =
// state[10] = k, mcts.py:62-64): the playout env seats exactly k players
__device__ __forceinline__ uint32_t league_mcs(int k, MtGen& gen, ByteBuf& buf, uint8_t* lds, const Board& b, const Hand& me,
                                               uint32_t n, u32x4 mem, int mpc, int mmax, bool* q6) {
    int32_t sum[kHand], cnt[kHand];
    switch (k) {
        case 2: return mcs_decide_exact<2>(gen, buf, lds, b, me, n, mem, mpc, mmax, sum, cnt, q6);
        case 3: return mcs_decide_exact<3>(gen, buf, lds, b, me, n, mem, mpc, mmax, sum, cnt, q6);
        case 4: return mcs_decide_exact<4>(gen, buf, lds, b, me, n, mem, mpc, mmax, sum, cnt, q6);
        case 5: return mcs_decide_exact<5>(gen, buf, lds, b, me, n, mem, mpc, mmax, sum, cnt, q6);
        default: return mcs_decide_exact<6>(gen, buf, lds, b, me, n, mem, mpc, mmax, sum, cnt, q6);
    }
}

template <int N>
__global__ __launch_bounds__(kBlock) void k_league_step(DevState s, LeagueStepArgs a) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[kBlock * kDealStride];
    const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= s.B) return;
    uint8_t* mine = lds + threadIdx.x * kDealStride;
    const int64_t B = s.B, DN = s.B * N;
    Game<N> G;
    load_game<N>(s, g, G);
    uint32_t lg = s.lgs[g];
    const uint32_t k = lg & 15u;
    // external seats first (no stream draws): an illegal card leaves the game untouched
    int bad = -1;
    uint32_t card[N], idx[N], pen[N];
#pragma unroll
    for (int p = N - 1; p >= 0; p--) {
        card[p] = 0xFFu, idx[p] = 0u;
        if ((uint32_t)p >= k) continue;
        const uint32_t agent = (lg >> (4 + 4 * p)) & 15u;
        if (((a.kinds >> (4 * agent)) & 15u) != (uint64_t)SN_AGENT_EXTERNAL) continue;
        const int32_t c = a.actions ? a.actions[g * N + p] : -1;
        const int kk = (c >= 0 && c < s.C) ? hand_find(G.hand[p], (uint32_t)c) : -1;
        if (kk < 0) bad = p;
        idx[p] = (uint32_t)max(kk, 0);
    }
    if (G.n == 0u) bad = 0;
    if (a.invalid) a.invalid[g] = bad;
    const int32_t pf = s.lpf ? s.lpf[g] : 0;
    if (pf) s.lpf[g] = 0;
    if (bad >= 0) return;
    if (pf) {  // k_league_mcs drew this slot's step: its non-external seats' cards
#pragma unroll
        for (int p = 0; p < N; p++) {
            if ((uint32_t)p >= k) continue;
            const uint32_t agent = (lg >> (4 + 4 * p)) & 15u;
            if (((a.kinds >> (4 * agent)) & 15u) == (uint64_t)SN_AGENT_EXTERNAL) continue;
            idx[p] = (uint32_t)max(hand_find(G.hand[p], (uint32_t)s.lpc[g * N + p]), 0);
        }
    }
    MtGen gen;
    ByteBuf buf;
    if (!pf) RngOf<RNG_NUMPY_MT>::load(s, g, gen, buf);
    int32_t status = (pf >> 1) & 1;
#pragma unroll
    for (int p = 0; p < N; p++) {  // GameSession.play_game: agents in seat order (play.py:38-41)
        if ((uint32_t)p >= k) continue;
        if (pf) {
            card[p] = hand_get(G.hand[p], idx[p]);
            continue;
        }
        const uint32_t agent = (lg >> (4 + 4 * p)) & 15u;
        const uint32_t kind = (uint32_t)((a.kinds >> (4 * agent)) & 15u);
        if (kind == SN_AGENT_RANDOM) {
            idx[p] = rng_interval(gen, buf, G.n - 1u);
        } else if (kind == SN_AGENT_MCS) {
            const int64_t dn = g * N + p;
            u32x4 mem = {s.lmem[dn], s.lmem[DN + dn], s.lmem[2 * DN + dn], s.lmem[3 * DN + dn]};
            mem = memorize(mem, G.n, (uint32_t)kMaxCards, G.hand[p], G.b);  // mcts.py:47-49, 62-73
            s.lmem[dn] = mem.x, s.lmem[DN + dn] = mem.y, s.lmem[2 * DN + dn] = mem.z, s.lmem[3 * DN + dn] = mem.w;
            if (G.n == 1u) {
                idx[p] = 0u;  // mcts.py:52-53: the last card, no search
            } else {
                bool q6 = false;
                const uint32_t c = league_mcs((int)k, gen, buf, mine, G.b, G.hand[p], G.n, mem, a.mpc[agent], a.mmax[agent], &q6);
                if (q6) status |= 1;
                idx[p] = (uint32_t)hand_find(G.hand[p], c);
            }
        }
        card[p] = hand_get(G.hand[p], idx[p]);
    }
#pragma unroll
    for (int p = 0; p < N; p++)
        if ((uint32_t)p < k) hand_del(G.hand[p], idx[p]);
    resolve<N, true>(G.b, card, pen);  // absent seats (card 0xFF) play nothing
#pragma unroll
    for (int p = 0; p < N; p++) {
        G.score[p] += (int32_t)pen[p];
        if (a.rewards) a.rewards[g * N + p] = -(int32_t)pen[p];
        if (a.played) a.played[g * N + p] = ((uint32_t)p < k) ? (int32_t)card[p] : -1;
    }
    G.n -= 1u;
    if (G.n == 0u) {
        // Tournament.score_game's input (session.results[0]), then the next
        // play_game: _choose_players, GameSession, env.reset (tournament.py:132-177)
        if (a.records) {
            int32_t* rec = a.records + g * (1 + N);
            rec[0] = (int32_t)lg;
#pragma unroll
            for (int p = 0; p < N; p++) rec[1 + p] = -G.score[p];
        }
#pragma unroll
        for (int p = 0; p < N; p++) s.sum_res[(int64_t)p * B + g] -= G.score[p];
        s.episodes[g] += 1;
        // the slot's next game (seats, then the deal) starts with the next
        // sn_reset, so the roster may change in between (Tournament.evolve)
    }
    if (a.status) a.status[g] |= status;
    store_game<N>(s, g, G);
    if (!pf) RngOf<RNG_NUMPY_MT>::store(s, g, gen, buf);
}

// One wave per slot whose game seats an MCSAgent this step (n >= 2): the
// slot's draws in seat order -- DrunkHamster seats' legal[random_interval(n-1)],
// MCS seats' whole searches (sechs_mcs_wave.h) -- on its numpy stream, the
// cards to lpc for k_league_step, which then resolves the step.
template <int N>
__global__ __launch_bounds__(64) void k_league_mcs(DevState s, LeagueStepArgs a) {
    __shared__ WmcsLds L;
    const int64_t g = blockIdx.x;
    const uint32_t lane = threadIdx.x;
    const uint32_t lg = s.lgs[g], k = lg & 15u;
    bool any = false;
    for (uint32_t p = 0; p < k; p++)
        any |= ((a.kinds >> (4 * ((lg >> (4 + 4 * p)) & 15u))) & 15u) == (uint64_t)SN_AGENT_MCS;
    if (!any) return;
    Game<N> G;
    load_game<N>(s, g, G);
    if (G.n < 2u) return;  // the last card: no search (mcts.py:52-53), k_league_step plays it
    const int64_t DN = s.B * N;
    WaveMt m{L.st, L.stage, 0u, 0u, 0u, 0u, false, nullptr};
    wmt_load(m, s.mt + g * kMtN, s.mt_pos[g], lane);
    int32_t q6s = 0;
    for (uint32_t p = 0; p < k; p++) {  // GameSession.play_game: agents in seat order (play.py:38-41)
        Hand hp = G.hand[0];  // seat p's hand by a select chain (a runtime index would keep G in scratch)
#pragma unroll
        for (int j = 1; j < N; j++) hp = (p == (uint32_t)j) ? G.hand[j] : hp;
        const uint32_t agent = (lg >> (4 + 4 * p)) & 15u;
        const uint32_t kind = (uint32_t)((a.kinds >> (4 * agent)) & 15u);
        uint32_t card = 0xFFu;
        if (kind == SN_AGENT_RANDOM) {
            const uint32_t mx = G.n - 1u;
            wmt_draws(m, 1u, [&](uint32_t) -> uint32_t { return mx; }, L.dr, lane);
            card = hand_get(hp, L.dr[0]);
        } else if (kind == SN_AGENT_MCS) {
            const int64_t dn = g * N + p;
            u32x4 mem = {s.lmem[dn], s.lmem[DN + dn], s.lmem[2 * DN + dn], s.lmem[3 * DN + dn]};
            mem = memorize(mem, G.n, (uint32_t)kMaxCards, hp, G.b);  // mcts.py:47-49, 62-73
            if (lane == 0u) s.lmem[dn] = mem.x, s.lmem[DN + dn] = mem.y, s.lmem[2 * DN + dn] = mem.z, s.lmem[3 * DN + dn] = mem.w;
            bool q6 = false;
            const int mpc = a.mpc[agent], mmax = a.mmax[agent];
            switch (k) {  // the playouts seat the game's k players (mcts.py:62-64)
                case 2: card = wmcs_decide_inl<2>(m, L, G.b, hp, G.n, mem, mpc, mmax, &q6, lane); break;
                case 3: card = wmcs_decide_inl<3>(m, L, G.b, hp, G.n, mem, mpc, mmax, &q6, lane); break;
                case 4: card = wmcs_decide_inl<4>(m, L, G.b, hp, G.n, mem, mpc, mmax, &q6, lane); break;
                case 5: card = wmcs_decide_inl<5>(m, L, G.b, hp, G.n, mem, mpc, mmax, &q6, lane); break;
                default: card = wmcs_decide_inl<6>(m, L, G.b, hp, G.n, mem, mpc, mmax, &q6, lane); break;
            }
            q6s |= q6 ? 1 : 0;
        }
        if (lane == 0u) s.lpc[g * N + p] = (int32_t)card;
    }
    wmt_store(m, s.mt + g * kMtN, s.mt_pos + g, s.mt0 + g, lane);
    if (lane == 0u) s.lpf[g] = 1 | (q6s << 1);
}

// ============================================================================
// C ABI
// ============================================================================
extern "C" {

sn_status sn_league_agents(sn_env* e, const int32_t* kinds, const int32_t* mc_per_card, const int32_t* mc_max) {
    if (!e || !kinds) return set_error(SN_EINVAL, "NULL argument");
    DevState& s = e->s;
    if (!s.lg_K) return set_error(SN_EINVAL, "not a tournament handle (sn_league_config)");
    bool mcs = false;
    for (int i = 0; i < s.lg_K; i++) {
        if (kinds[i] < SN_AGENT_RANDOM || kinds[i] > SN_AGENT_EXTERNAL) return set_error(SN_EINVAL, "unknown agent kind");
        const int mpc = mc_per_card ? mc_per_card[i] : 10, mmax = mc_max ? mc_max[i] : 100;
        if (kinds[i] == SN_AGENT_MCS) {
            if (mpc < 0 || mmax < 0) return set_error(SN_EINVAL, "mc_per_card and mc_max must be >= 0");
            mcs = true;
        }
        e->lg_kind[i] = kinds[i], e->lg_mpc[i] = mpc, e->lg_mmax[i] = mmax;
    }
    if (mcs && s.rng_mode != SN_RNG_NUMPY_MT)
        return set_error(SN_EINVAL, "MCSAgent seats draw from numpy MT19937 streams (rng_mode numpy)");
    if (mcs && !s.lmem) {  // card memory [4][B*N], then k_league_mcs's cards [B*N] and flags [B]
        HIP_TRY(hipSetDevice(e->device));
        const size_t BN = (size_t)s.B * s.N, bytes = sizeof(uint32_t) * (5 * BN + (size_t)s.B);
        if (hipMalloc((void**)&s.lmem, bytes) != hipSuccess) return set_error(SN_ENOMEM, "league card memory");
        HIP_TRY(hipMemset(s.lmem, 0, bytes));
        s.lpc = (int32_t*)(s.lmem + 4 * BN);
        s.lpf = s.lpc + BN;
    }
    return SN_OK;
}

sn_status sn_league_step(sn_env* e, const int32_t* actions, int32_t* rewards, int32_t* played, int32_t* records,
                         int32_t* invalid, int32_t* status, void* stream) {
    if (!e) return set_error(SN_EINVAL, "env is NULL");
    DevState& s = e->s;
    if (!s.lg_K) return set_error(SN_EINVAL, "not a tournament handle (sn_league_config)");
    if (s.rng_mode != SN_RNG_NUMPY_MT) return set_error(SN_EUNSUPPORTED, "sn_league_step plays numpy-MT tournament handles");
    if (e->lg_phase < 0) return set_error(SN_EINVAL, "start the slots' games with sn_reset (seat draw + deal)");
    if (s.N < 2 || s.N > kLeagueMaxPlayers) return set_error(SN_EINVAL, "tournament handles seat 2..6 players");
    bool ext = false, mcs = false;
    LeagueStepArgs a{};
    for (int i = 0; i < s.lg_K; i++) {
        a.kinds |= (uint64_t)(e->lg_kind[i] & 15) << (4 * i);
        a.mpc[i] = e->lg_mpc[i], a.mmax[i] = e->lg_mmax[i];
        ext |= e->lg_kind[i] == SN_AGENT_EXTERNAL;
        mcs |= e->lg_kind[i] == SN_AGENT_MCS;
    }
    if (ext && !actions) return set_error(SN_EINVAL, "the league has external agents: actions must be given");
    if (mcs && !s.lmem) return set_error(SN_EINVAL, "sn_league_agents did not allocate the MCS card memory");
    hipStream_t st = (hipStream_t)stream;
    if (sn_pipe_sync(e, st) != SN_OK) return SN_EHIP;  // the step draws from the plain MT state
    a.actions = actions, a.rewards = rewards, a.played = played, a.records = records, a.invalid = invalid;
    a.status = status;
    if (mcs && kHand - e->lg_phase >= 2) {  // the MCS seats' searches, one wave per slot
        switch (s.N) {
            case 2: hipLaunchKernelGGL((k_league_mcs<2>), dim3((unsigned)s.B), dim3(64), 0, st, s, a); break;
            case 3: hipLaunchKernelGGL((k_league_mcs<3>), dim3((unsigned)s.B), dim3(64), 0, st, s, a); break;
            case 4: hipLaunchKernelGGL((k_league_mcs<4>), dim3((unsigned)s.B), dim3(64), 0, st, s, a); break;
            case 5: hipLaunchKernelGGL((k_league_mcs<5>), dim3((unsigned)s.B), dim3(64), 0, st, s, a); break;
            default: hipLaunchKernelGGL((k_league_mcs<6>), dim3((unsigned)s.B), dim3(64), 0, st, s, a); break;
        }
        HIP_TRY(hipGetLastError());
    }
    switch (s.N) {
        case 2: hipLaunchKernelGGL((k_league_step<2>), dim3(grid_for(s.B)), dim3(kBlock), 0, st, s, a); break;
        case 3: hipLaunchKernelGGL((k_league_step<3>), dim3(grid_for(s.B)), dim3(kBlock), 0, st, s, a); break;
        case 4: hipLaunchKernelGGL((k_league_step<4>), dim3(grid_for(s.B)), dim3(kBlock), 0, st, s, a); break;
        case 5: hipLaunchKernelGGL((k_league_step<5>), dim3(grid_for(s.B)), dim3(kBlock), 0, st, s, a); break;
        default: hipLaunchKernelGGL((k_league_step<6>), dim3(grid_for(s.B)), dim3(kBlock), 0, st, s, a); break;
    }
    HIP_TRY(hipGetLastError());
    e->lg_phase = (e->lg_phase + 1 == kHand) ? -1 : e->lg_phase + 1;  // games over: the next ones start at sn_reset
    e->phase = -1;
    return SN_OK;
}

}  // extern "C"

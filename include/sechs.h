/*
 * sechs.h -- C ABI of libsechs.so, the MI355X-native vectorised 6 nimmt!
 * engine (environment + random-policy self-play + Monte-Carlo search).
 *
 * The reference (coolo/rl-6-nimmt) is pure Python and has no FFI: its hot
 * path sits behind duck-typed Python interfaces.  Each entry point below
 * names the reference interface it replaces; the Python package
 * rl-6-nimmt_amd/rl_6_nimmt binds them with ctypes and
 * re-exposes the reference API (SechsNimmtEnv, GameSession, Tournament,
 * DrunkHamster, MCSAgent, ...).
 *
 * Conventions
 *  - No exceptions cross the ABI: every call returns sn_status; the text of
 *    the last error on the calling thread is sn_last_error().
 *  - The engine owns its device state.  The caller owns every I/O buffer;
 *    I/O pointers are DEVICE pointers (e.g. torch.Tensor.data_ptr() of a
 *    cuda tensor) unless the parameter name ends in _host.
 *  - `stream` is a hipStream_t (NULL = the default stream).  Calls only
 *    enqueue work; they never synchronise the stream, except those marked
 *    [sync] (host-side state exchange).
 *  - One handle per device; no internal locking.  Several handles on
 *    several GPUs (one process per GPU) are independent.
 *  - Game g of a handle has the global id game_offset + g; every random
 *    stream is keyed by the global id, so results do not depend on how the
 *    games are sharded over handles / ranks.
 *  - Layouts are row-major, game-major: obs [B][N][obs_stride] etc.
 */
#ifndef SECHS_H
#define SECHS_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct sn_env sn_env; /* opaque */

typedef enum {
    SN_OK = 0,
    SN_EINVAL = 1,       /* bad argument (reference: AssertionError, env.py:19-21,67) */
    SN_EHIP = 2,         /* HIP runtime error */
    SN_ENOMEM = 3,       /* device allocation failed */
    SN_EUNSUPPORTED = 4, /* valid in the reference but not built here */
    SN_ERNG = 5,         /* a pipelined numpy-MT draw ran past the twisted words (sticky: every
                            rollout of this handle since then is invalid; see sn_pipe_errors) */
} sn_status;

/* random word sources; both drive numpy's legacy masked-rejection
   random_interval, so the draw structure is the reference's */
enum {
    SN_RNG_PHILOX = 0,   /* counter-based Philox4x32-10 keyed (seed, global game id) */
    SN_RNG_NUMPY_MT = 1, /* numpy legacy RandomState per game, seeded seed + global game id:
                            game g replays np.random.seed(seed+g) + GameSession(DrunkHamster x N) */
};

/* observation element types for sn_obs */
enum { SN_I8 = 1, SN_I16 = 2, SN_I32 = 3, SN_I64 = 4, SN_F32 = 5 };

/* sn_rollout / sn_step flags */
enum {
    SN_AUTO_RESET = 1,       /* a finished game is re-dealt at once from its own stream */
    SN_NO_SUMMARIES = 2,     /* obs without the 12 row summaries (include_summaries=False) */
};

const char* sn_last_error(void);
const char* sn_version(void);

/* SechsNimmtEnv.__init__ (env.py:16-41) for B games at once.
   num_players 1..10, num_cards 10*N+4 .. 104 (env.py:19-21; cards >= 104
   fail the reference's own _card_value assertion, env.py:228).
   num_rows / threshold are fixed at the reference defaults 4 / 6. */
sn_status sn_create(sn_env** out, int device, int64_t num_games, int num_players, int num_cards, uint64_t seed,
                    uint64_t game_offset, int rng_mode);
sn_status sn_destroy(sn_env* env);
sn_status sn_info(const sn_env* env, int64_t* num_games, int* num_players, int* num_cards, int* rng_mode);

/* env.py:43-51 reset() -> _deal() (:99-112).  decks == NULL: every game
   shuffles arange(C) from its own stream (np.random.shuffle); else decks
   is [B][C] uint8, one permutation per game.  Scores are zeroed. */
sn_status sn_reset(sn_env* env, const uint8_t* decks, void* stream);

/* env.py:53-62 reset_to(board, hands): board [B][4][6] int8 (row cards,
   -1 padded, 1..5 cards per row), hands [B][N][10] int8 (-1 padded, every
   seat holding the same count).  Scores are zeroed.  Inputs are copied. */
sn_status sn_reset_to(sn_env* env, const int8_t* board, const int8_t* hands, void* stream);

/* env.py:64-77 step(action).  actions [B][N] int32 (NULL = the in-kernel
   DrunkHamster policy, agents/random.py:8-10, drawn in seat order from each
   game's stream).  Outputs: rewards [B][N] int32 (<= 0), done [B] uint8,
   invalid [B] int32 = first seat whose card is not in its hand or -1 (the
   reference raises InvalidMoveException, env.py:114-118; the game is left
   untouched).  Any output may be NULL.  flags: SN_AUTO_RESET. */
sn_status sn_step(sn_env* env, const int32_t* actions, int32_t* rewards, uint8_t* done, int32_t* invalid, int flags,
                  void* stream);

/* Fused self-play: `steps` env-steps of every game with the DrunkHamster
   policy in one launch (GameSession.play_game, play.py:23-75, looped with
   auto-reset).  Per-step outputs, each optional (NULL):
     rewards [steps][B][N] int32, done [steps][B] uint8,
     actions [steps][B][N] uint8,
     obs     [steps][B][N][obs_stride] int8: the observation each seat acts
             on (env.py:174-212, pre-action), zero-padded to obs_stride >= L.
   flags: SN_AUTO_RESET (required when steps run past a game's end),
          SN_NO_SUMMARIES. */
sn_status sn_rollout(sn_env* env, int steps, int32_t* rewards, uint8_t* done, uint8_t* actions, int8_t* obs,
                     int obs_stride, int flags, void* stream);

/* env.py:174-212 _create_states: obs [B][N][obs_stride] of `dtype`
   (L = 47, or 35 with SN_NO_SUMMARIES; padding is zero). */
sn_status sn_obs(sn_env* env, void* obs, int dtype, int obs_stride, int flags, void* stream);
/* legal_actions (env.py:209): hands [B][N][10] int8 ascending, -1 padded */
sn_status sn_hands(sn_env* env, int8_t* hands, void* stream);
/* the board (env.py:30,191-194): [B][4][6] int8, -1 padded */
sn_status sn_board(sn_env* env, int8_t* board, void* stream);
/* _scores (env.py:32,167): [B][N] int32 penalties so far this episode */
sn_status sn_scores(sn_env* env, int32_t* scores, void* stream);
/* episode accumulators for auto-reset play (GameSession.results,
   play.py:74): sum over finished episodes of the final scores (-penalty)
   [B][N] int32, and the finished-episode count [B] int32.  Either may be NULL. */
sn_status sn_results(sn_env* env, int32_t* sum_results, int32_t* episodes, void* stream);
sn_status sn_clear_results(sn_env* env, void* stream);

/* numpy global-RNG bridge for the drop-in scalar API [sync]: export /
   import game g's MT19937 state in np.random.get_state() form
   (key_host[624] uint32, pos_host in 0..624). */
sn_status sn_mt_get(sn_env* env, int64_t game, uint32_t* key_host, int32_t* pos_host);
sn_status sn_mt_set(sn_env* env, int64_t game, const uint32_t* key_host, int32_t pos);
/* philox word counter of game g [sync] */
sn_status sn_philox_counter(sn_env* env, int64_t game, uint64_t* counter_host);

/* Tuning knobs of the numpy-compat DrunkHamster rollout (results never
   depend on them; the tests run both ways):
     SN_OPT_RING_WORDS   words each game's stream is twisted ahead per
                         launch by k_mt_prep (multiple of 64, 64..512;
                         0 = no ring, k_play twists lazily per lane).
                         Default 256 for N <= 4, else 512.
     SN_OPT_CHUNK_STEPS  env-steps per k_mt_prep-fed launch (>= 1, default 10).
     SN_OPT_PIPELINE     1 (default): DrunkHamster rollouts in numpy mode keep
                         each stream twisted ~600 words ahead with k_mt_ahead
                         on a side stream, concurrently with the previous
                         launch's k_play (N <= 6); 0: the paths above.
     SN_OPT_TIMING       n > 0: record HIP events around the next n
                         pipelined k_play / k_mt_ahead launches, each on the
                         stream it runs on (read with sn_kernel_times);
                         0 (default): off.
     SN_OPT_PIPE_GPW     games per k_play wave on the pipelined path: 64
                         (one per lane) or 32 (half the LDS per wave, two
                         waves per SIMD).
     SN_OPT_PIPE_LEAD    words k_mt_ahead keeps twisted past the consumer
                         (64..600, default 600).  TEST KNOB: below 600 the
                         overrun bound of sn_pipe_errors no longer holds;
                         it exists to exercise the SN_ERNG path.
     SN_OPT_PLAY_SPLIT   role-split k_play (producer waves decode every random
                         decision into LDS beside the play waves) for in-kernel
                         DrunkHamster rollouts of a Philox handle whose games
                         are in lockstep (after sn_reset; N <= 4, auto-reset):
                         1 (default) or 0 (never).  Measured (65 536 x 4p):
                         74 -> 59 us per 10 env-steps.  Numpy-compat handles
                         always use the pipelined one-wave k_play.
     SN_OPT_PLAY_QUAD    removed (round 6): k_play_quad, four lanes per game,
                         measured slower; SN_EUNSUPPORTED.
     SN_OPT_TWIST_ROUND  1 (default): the pipelined twist-ahead k_mt_ahead
                         twists whole MT19937 rounds (each old word read
                         once, each new word written once: 8 instead of 12
                         B of MT-state traffic per word); 0: exactly the
                         words the lead needs.  Same words either way.
     SN_OPT_TWIST_EVERY  K = 1 .. 5 (default 4): play launches in groups of
                         K; one k_mt_ahead beside the first launch of each
                         group twists 600 K words past the consumer (the
                         next 2K launches' draws), and that launch waits for
                         the twist of the group before only -- per group one
                         cross-stream wait and one record instead of one per
                         launch.
     SN_OPT_PIPE_FUSED   removed (round 6): the twist folded into k_play_quad,
                         measured slower; SN_EUNSUPPORTED.
     SN_OPT_PIPE_DEC     1 (default): pipelined numpy-compat DrunkHamster rollouts
                         with auto-reset of a plain handle of N <= 4 whose games
                         are in lockstep (after sn_reset) decode ahead: on a
                         second side stream, concurrent with each group's
                         twist (reading the words the twist before produced),
                         k_decode walks every game's ring a group ahead of the
                         play launches and writes one record per episode
                         (its draws, the next deal's sorted hands and rows, the
                         stream offsets), and k_play plays from the records
                         with no RNG work; 0: k_play draws from the ring itself.
                         Same words, same outputs, same exported numpy states.
     SN_OPT_TWIST_SKIP   TEST KNOB: 1 = every steady twist after the first
                         group's twists nothing, so the default schedule
                         runs its ring dry (the SN_ERNG / sn_pipe_errors
                         path); 0 (default): off.
   A pipelined (numpy-compat) rollout records its ordering event on the
   caller's stream before it returns; every later call waits on that event
   (also on the same stream), so the caller may destroy the stream after
   the call. */
enum { SN_OPT_RING_WORDS = 1, SN_OPT_CHUNK_STEPS = 2, SN_OPT_PIPELINE = 3, SN_OPT_TIMING = 4, SN_OPT_PIPE_GPW = 5,
       SN_OPT_PIPE_LEAD = 6, SN_OPT_PLAY_SPLIT = 7, SN_OPT_PLAY_QUAD = 8, SN_OPT_TWIST_ROUND = 9,
       SN_OPT_TWIST_EVERY = 10, SN_OPT_PIPE_FUSED = 11, SN_OPT_TWIST_SKIP = 12, SN_OPT_PIPE_DEC = 13 };
sn_status sn_set_option(sn_env* env, int option, int value);
/* pipelined rollouts whose draws ran past the twisted words (must be 0; a
   nonzero count means those games' draws are wrong) [sync].  The count is
   also mirrored asynchronously into pinned host memory after every
   pipelined rollout: sn_rollout returns SN_ERNG once a completed rollout
   has counted one (sticky for the handle). */
sn_status sn_pipe_errors(sn_env* env, uint32_t* count);
/* mean launch duration (ms) of the pipelined k_play and k_mt_ahead launches
   recorded since SN_OPT_TIMING was set; *n = launches recorded [sync] */
sn_status sn_kernel_times(sn_env* env, float* play_ms, float* ahead_ms, int32_t* n);
/* the same, and the mean duration of the k_decode launches (decode-ahead
   mode; 0 if none ran) [sync] */
sn_status sn_kernel_times_dec(sn_env* env, float* play_ms, float* ahead_ms, float* decode_ms, int32_t* n);
/* Diagnostics (no reference counterpart): shader-clock cycles every k_play
   wave spent per phase of its step loop since the last call, summed over
   waves -- out[0..10] = prologue, obs, draws, resolve, output stores, deck
   shuffle targets, epilogue, hand sorting, deck shuffle swaps, and (role-
   split play waves) the waits at the two barriers; out[11..18] = the split
   kernel's producer waves: draws, barrier 1, shuffle targets, swaps, hands,
   later draws, barrier 2, state store, twist-ahead; out[20] = play waves,
   out[21] = producer waves.  Only the libsechs_prof.so build
   (-DSECHS_PHASE_PROF) records them; the product build returns
   SN_EUNSUPPORTED [sync]. */
sn_status sn_debug_phases(uint64_t* out, int n);
/* k_puct_rollouts phase counters of a -DSECHS_PHASE_PROF build (diagnostics):
   out[0..4] = shader-clock cycles summed over waves in the state copy-in, the
   seat rows, the per-seat layer-1 MFMA, the candidate tiles and the step;
   out[7] = waves; read and cleared.  SN_EUNSUPPORTED in the product library. */
sn_status sn_debug_puct_phases(uint64_t* out, int n);
/* pipeline words to the host (tests, diagnostics) [sync]: what 0 = pabsc[slot]
   (consumer positions, slot kPipeSlots = the decoder's; B words), 1 =
   ptend[slot] (B words), 2 = decode-ahead record slot (kDecQuads x B 16-B
   pieces, piece-major).  No pipeline state is changed. */
sn_status sn_debug_pipe_words(sn_env* env, int what, int slot, uint32_t* out);
/* Device-side invariant checks (SN_DASSERT in sechs_device.h / sechs_env.hip:
   a played card is in its seat's hand, the cards of a step are distinct, a
   card goes to a row ending below it (or undercuts), rows hold 1..5 cards,
   a deal gives ten distinct cards per hand): violations counted since the
   last call, *first_line = the smallest source line that failed; the
   counters are cleared.  selftest != 0 first runs one deliberately failing
   check.  Only the libsechs_debug.so build (-DSECHS_DEBUG) has them; the
   product build returns SN_EUNSUPPORTED [sync]. */
sn_status sn_debug_failures(uint32_t* count, uint32_t* first_line, int selftest);

/* ---- One-game fast path (the scalar drop-in SechsNimmtEnv) ------------
   For a handle of B == 1: one kernel launch and one stream sync per call
   (host-memory arguments and results; pinned, device-mapped buffer inside
   the handle).  out_host: int32 [2 + 15N] = first illegal seat or -1
   (env.py:114-118; nothing changes then), done, rewards [N] (env.py:64-77),
   scores [N] (penalties so far), then the N observation rows as int8 bytes,
   48 per seat (47 used, env.py:174-212), then per seat the placement of its
   card for the debug trace (env.py:128,145,165): target row | undercut
   (_pick_row_to_replace) << 2 | scored (_score_row) << 3 | penalty << 8
   (all 0 after an illegal step or a reset). [sync] */
sn_status sn_step1(sn_env* env, const int32_t* actions_host, int32_t* out_host, int flags);
/* env.py:43-51 reset() drawing from the numpy legacy state (key, pos) given
   -- np.random.get_state() -- and returning the advanced state for
   np.random.set_state(); out_host as sn_step1 (invalid -1, rewards 0).
   numpy-compat handles only. [sync] */
sn_status sn_reset1(sn_env* env, const uint32_t* key_host, int32_t pos, uint32_t* key_out_host, int32_t* pos_out,
                    int32_t* out_host, int flags);

/* ---- Batched tournament (tournament.py:132-177) ------------------------
   A tournament handle plays one league game per game slot at a time: slot
   g is the reference's `np.random.seed(seed + game_offset + g); t =
   Tournament(min_players, max_players) over num_agents DrunkHamster
   agents; t.play_game() x games` -- every game first draws its seats
   (_choose_players: num_players = choice(range(min, max+1)), agents =
   choice(num_agents, num_players, replace=False)), then GameSession deals
   and plays it, all from the slot's own stream.  The handle's num_players
   is max_players; seats past a game's player count hold empty hands and
   play nothing.  In-kernel DrunkHamster seats only (the search agents play
   through the drop-in Tournament).  Elo (order dependent) is replayed on
   the host from the records (sn_elo_replay). */
/* turn a handle (num_players = max_players, 2..6) into a tournament of
   num_agents (max_players..16) agents; 0 agents turns it back.  The next
   sn_reset draws every slot's first seats and deals [sync]. */
sn_status sn_league_config(sn_env* env, int num_agents, int min_players, int max_players);
/* play steps/10 whole games per slot (auto-reset: each finished game's
   slot draws its next seats and deals).  records: [steps/10][B][1 + N]
   int32 per finished game: seats word (k | agent(seat p) << (4 + 4p)),
   then the N results (GameSession.results[0]: -penalties; 0 past k).
   rewards/done/actions/obs as sn_rollout (may be NULL). */
sn_status sn_league_rollout(sn_env* env, int steps, int32_t* rewards, uint8_t* done, uint8_t* actions, int8_t* obs,
                            int obs_stride, int32_t* records, void* stream);
/* the seats word of every slot's current game, [B] uint32 */
sn_status sn_league_seats(sn_env* env, uint32_t* out, void* stream);

/* Mixed leagues (run.py:20-40: DrunkHamster, MCSAgent, PUCTAgent,
   PUCTCustomedAgent, BatchedACERAgent seats).  sn_league_agents gives every
   agent of a tournament handle its kind (kinds[num_agents]; all
   SN_AGENT_RANDOM after sn_league_config):
     SN_AGENT_RANDOM    DrunkHamster, drawn in-kernel from the slot's stream
     SN_AGENT_MCS       MCSAgent(mc_per_card[a], mc_max[a]) (agents/mcts.py:17-188):
                        card memory and the reference-exact search on the
                        slot's numpy stream (numpy handles only)
     SN_AGENT_EXTERNAL  the caller plays the seat (the net agents: their
                        batched engines pick the card, sn_puct over the
                        handle's decision list, sn_puct.dec_list)
   mc_per_card / mc_max may be NULL (10 / 100, mcts.py:24-25).  Leagues with
   any non-RANDOM agent play with sn_league_step; all-RANDOM ones also with
   sn_league_rollout. [sync] */
enum { SN_AGENT_RANDOM = 0, SN_AGENT_MCS = 1, SN_AGENT_EXTERNAL = 2 };
sn_status sn_league_agents(sn_env* env, const int32_t* kinds_host, const int32_t* mc_per_card_host,
                           const int32_t* mc_max_host);
/* One env-step of every slot's current game (numpy handles; sn_reset then
   10 steps per game): seats in seat order as GameSession calls
   them (play.py:38-41) -- RANDOM and MCS seats draw from the slot's stream in
   the reference's exact order, EXTERNAL seats play actions [B][N] (checked
   against the hand, env.py:114-118).  A game that ends (every 10th step)
   writes records [B][1 + N] (seats word, GameSession.results[0]); the
   slots' next games start with sn_reset (seat draw, then deal:
   tournament.py:132-138), after any roster change.  Outputs (each may
   be NULL): rewards [B][N], played [B][N] (cards, -1 past k), invalid [B]
   (first seat whose external card is illegal, or -1: that slot's board,
   hands and scores are left as they were, but its RANDOM / MCS seats have
   already drawn this step from the slot's stream and an MCS seat's card
   memory has moved on -- the slot no longer follows the reference's stream
   and the caller must treat it as failed; the batched tournament raises right
   after such a step), status [B] |= 1 where an MCSAgent move got no playout
   (the reference raises IndexError there, quirk Q6). */
sn_status sn_league_step(sn_env* env, const int32_t* actions, int32_t* rewards, int32_t* played, int32_t* records,
                         int32_t* invalid, int32_t* status, void* stream);
/* Sequential multiplayer Elo over game records in the given order (host
   memory, no GPU): records [G][1 + max_players] int32 as sn_league_rollout
   writes them; elos [num_agents] float64 in/out (initial ratings in).
   Places are Tournament._compute_absolute_positions of the k results,
   ratings update by the multiplayer Elo of rl_6_nimmt/elo.py (multi_elo's
   scheme; parity unpinned: multi_elo is absent). */
sn_status sn_elo_replay(const int32_t* records_host, int64_t num_games, int max_players, int num_agents, double elo_k,
                        double* elos_host);

/* ---- Monte-Carlo search, MCSAgent (agents/mcts.py:17-188) ------------- */

/* Card memory of every seat (mcts.py:62-73), updated in place from the
   current position: at a hand of 10 it restarts as range(mcs_num_cards),
   then the own hand and every card on the board are removed.
   avail: [4][B*N] uint32 card sets (word-major, decision d = g*N + p). */
sn_status sn_mcs_memorize(sn_env* env, uint32_t* avail, int mcs_num_cards, void* stream);

/* Stratified Monte-Carlo search for every (game, seat) at once (BASELINE
   config 3): `rollouts` playouts per legal first move, opponents dealt from
   the seat's memory, every later move uniform (mcts.py:108-154).
   sums [B*N][10] int32 = summed return of the seat per first move (slots
   >= the hand size are 0).  Random words: Philox keyed (seed ^
   decision_step, game id, seat, move, playout).  rollouts: 64, 128, 192 or
   a multiple of 256. */
sn_status sn_mcs_rollouts(sn_env* env, const uint32_t* avail, int rollouts, uint64_t seed, uint32_t decision_step,
                          int32_t* sums, void* stream);
/* same, also writing every playout's return: playouts [B*N][10][rollouts] int32 (may be NULL) */
sn_status sn_mcs_rollouts_ex(sn_env* env, const uint32_t* avail, int rollouts, uint64_t seed, uint32_t decision_step,
                             int32_t* sums, int32_t* playouts, void* stream);

/* _choose_action_from_outcomes (mcts.py:156-165) with equal playout counts:
   actions [B][N] int32 = legal[argmax sums] (ties -> lowest card), legal[0]
   for a one-card hand, -1 for an empty hand. */
sn_status sn_mcs_choose(sn_env* env, const int32_t* sums, int32_t* actions, void* stream);

/* Reference-exact replay (numpy-MT env only): every game of the handle plays
   one whole GameSession game (reset + 10 steps) with seat p an
   MCSAgent(mc_per_card, mc_max) if bit p of mcs_seats is set, else a
   DrunkHamster, consuming the game's MT19937 stream in the reference's
   exact order.  actions / rewards [10][B][N] int32; status [B] = 1 where the
   reference would have raised IndexError (quirk Q6, a move without playouts). */
sn_status sn_mcs_play_exact(sn_env* env, uint32_t mcs_seats, int mc_per_card, int mc_max, int32_t* actions,
                            int32_t* rewards, int32_t* status, void* stream);

/* Reference-exact MCSAgent._mcts for D independent decisions (one lane
   each), for the drop-in agent.  Device buffers: board [D][4][6] int8 (-1
   pad), hand [D][10] int8 (the legal actions, -1 pad), avail [D][4] uint32
   card memory, mt_keys [D][624] + mt_pos [D]: numpy-form MT19937 states
   (np.random.get_state()[1:3]) advanced in place.  actions [D] int32: the
   chosen card, or -(card)-2 when quirk Q6 applies; sums / counts [D][10]
   (optional) = per-move playout sums and counts. */
sn_status sn_mcs_decide_exact(int device, int64_t num_decisions, int num_players, const int8_t* board,
                              const int8_t* hand, const uint32_t* avail, int mc_per_card, int mc_max,
                              uint32_t* mt_keys, int32_t* mt_pos, int32_t* actions, int32_t* sums, int32_t* counts,
                              void* stream);

/* ---- "Alpha0.5" PUCT search, PUCTAgent / PolicyMCSAgent (mcts.py:191-323) ----
   The rollouts of one decision are a dependent chain (each root choice reads
   the outcomes so far), so a batch advances rollout `rollout` of every
   decision by one step per call; the policy MLP runs between the calls in
   PyTorch-ROCm.  Per decision d (game g = d / M, seat = the (d % M)-th set
   bit of seats_mask, M = popcount):
     sn_puct_root_rows  rows [D*n][48] (bf16 or f32): [legal[k], obs] normalised
                        as SechsNimmtStateNormalization (preprocessing.py:12-57)
     sn_puct_init       root_probs = softmax(root logits [D*n] f32); clears stats
     for rollout r:  sn_puct_deal (opponents from the memory, mcts.py:116-127)
       for t < n:    sn_puct_rows (rows [D*N*(n-t)][48] of every rollout seat),
                     MLP -> logits [D*N*(n-t)] f32, sn_puct_step (PUCT at the
                     root / policy samples elsewhere, env step, backup at the end)
     sn_puct_choose     actions [B][N] int32 of the deciding seats = best mean
   Buffers (device, caller-owned): rollouts [D][48] i32, stats [D][24] i32,
   hist [D][172] i32, root_probs [D][10] f32. */
typedef struct {
    uint32_t seats_mask;   /* deciding seats (bit p = seat p) */
    int n;                 /* hand size at the root (all games in lockstep) */
    int puct_root;         /* 1: PUCTAgent (PUCT at the root), 0: PolicyMCSAgent (sampled root) */
    double c_puct;         /* mcts.py:267, default 2.0 */
    uint64_t seed;
    uint32_t step;         /* decision counter, mixed into the Philox key */
    uint32_t rollout;      /* rollout index r */
    const uint32_t* avail; /* [4][B*N] card memory from sn_mcs_memorize */
    int32_t* rollouts;
    int32_t* stats;
    int32_t* hist;
    float* root_probs;
    const uint32_t* step_dev; /* NULL, or the decision counter in device memory (overrides `step`):
                                 lets one captured hipGraph of a decision's launches serve every decision */
    const int32_t* dec_list;  /* NULL (seats_mask), or num_dec decisions g * N + p in device memory: one
                                 agent's seats of a tournament handle (required there); a game of k < N
                                 players then rolls out k seats (obs N field k, mcts.py:62-64) and writes
                                 dummy rows for the absent seats */
    int64_t num_dec;
    int32_t logit_stride;     /* sn_puct_step: elements between consecutive candidates' logits (0 or 1: packed) */
    int32_t logit_bf16;       /* sn_puct_step: the logits are bf16 (e.g. a head GEMM padded to 16 outputs,
                                 logit_stride 16), not f32 */
} sn_puct;

sn_status sn_puct_root_rows(sn_env* env, const sn_puct* q, void* rows, int bf16, void* stream);
sn_status sn_puct_init(sn_env* env, const sn_puct* q, const float* root_logits, void* stream);
sn_status sn_puct_deal(sn_env* env, const sn_puct* q, void* stream);
/* sn_puct_deal for rollouts r0 .. r0 + nr - 1 in one launch: rollout r's
   initial state at ro_out + ((r - r0) * num_decisions + d) * 48 int32 (the
   layout of sn_puct.rollouts); point sn_puct.rollouts at rollout r's slice
   and run its steps there -- the same states, dealt with nr x D lanes. */
sn_status sn_puct_deal_batch(sn_env* env, const sn_puct* q, int r0, int nr, void* ro_out, void* stream);
/* Rollouts r0 .. r0 + nr - 1 of every decision in one launch, from the
   states sn_puct_deal_batch dealt into ro_base: one wave per group of up to
   32 / L decisions (L = N rounded up to 4 or 8; the library picks the
   smallest group that keeps the launch's rounds over its waves at their
   minimum) runs every step (sn_puct_mlp_seats' rows, MFMA layer 1 + 2 and
   head into logits in LDS, then sn_puct_step's seat-lane step) of each
   rollout in order -- the same values as the launch-per-step loop (3 <= N
   <= 8; weights as sn_puct_mlp_seats). */
sn_status sn_puct_rollouts(sn_env* env, const sn_puct* q, int r0, int nr, void* ro_base, const void* w1s,
                           const float* w1c, const void* w2, const float* head, void* stream);
sn_status sn_puct_rows(sn_env* env, const sn_puct* q, int n_cur, void* rows, int bf16, void* stream);
sn_status sn_puct_step(sn_env* env, const sn_puct* q, const float* logits, int t, int n_cur, void* stream);
/* Rollout MLP in one kernel per rollout step, for MultiHeadedMLP(48, (H, H2),
   (1,)) in bf16, H <= 111, H2 <= 127 -- the reference's policy net,
   utils/nets.py:100-132, evaluated in mcts.py:219-228: persistent
   workgroups loop over groups of 64 rollout seats, build their [0, obs, 1]
   rows in LDS (the card slot 0), multiply them by w1s [128][64] bf16 (the
   [W1 | b1 | 0] rows, 1 at (H, 48): the ones feature) on MFMA into base,
   then per candidate row h1[k] = bf16(relu(base[seat][k] + card * w1c[k]))
   (w1c = W1[:, 0] f32, 112 entries), layer 2 against w2 [128][112] bf16 =
   [W2 | b2 | 0] rows (+ the ones pass-through row H2), ReLU + bf16, and the
   head [128] f32 = [wh | bh | 0]: logits [D*N*n_cur] f32, packed, for
   sn_puct_step (logit_stride 1, logit_bf16 0).  No activation reaches HBM.
   w1s, w1c, w2, head 16-B aligned.  (The round-4 GEMM form -- seat rows, a
   PyTorch GEMM, a tile kernel -- the round-3 feature-major split and the
   round-5 per-candidate MFMA layer 1 measured slower and were removed in
   round 6; other nets take sn_puct_rows + the module's own forward.) */
sn_status sn_puct_mlp_seats(sn_env* env, const sn_puct* q, int n_cur, const void* w1s, const float* w1c, const void* w2,
                            const float* head, float* logits, void* stream);
/* best_index [D] (optional): index of the chosen card in the root legal list */
sn_status sn_puct_choose(sn_env* env, const sn_puct* q, int32_t* actions, int32_t* best_index, void* stream);
/* PUCTCustomedAgent (agents/mcts.py:325-451, replaces _mcts /
   _play_out_with_NN / _choose_action_mc_func :356-395): no rollouts.  heads
   [D*n][2] f32 = the 2-head net (policy logit, value) on the
   sn_puct_root_rows rows; per decision: best = first argmax of the values,
   actions [B][N] (deciding seats) = legal[best], best_index [D],
   log_prob [D] = log softmax(policy)[best], value [D] = values[best] (the
   "outcome" learn() regresses).  Optional outputs may be NULL. */
sn_status sn_pcv_choose(sn_env* env, const sn_puct* q, const float* heads, int32_t* actions, int32_t* best_index,
                        float* log_prob, float* value, void* stream);
/* BatchedReinforceAgent.forward (agents/policy.py:137-156) for every
   deciding seat of q->seats_mask at hand size q->n: logits [D*n] f32 = the
   policy MLP on the sn_puct_root_rows rows; samples Categorical(softmax)
   with Philox (key q->seed ^ q->step; torch's CPU generator is not
   reproducible on the device), actions [B][N] (deciding seats) = legal[k],
   index [D] = k, log_prob [D], entropy [D] (optional, may be NULL). */
sn_status sn_policy_sample(sn_env* env, const sn_puct* q, const float* logits, int32_t* actions, int32_t* index,
                           float* log_prob, float* entropy, void* stream);
/* _compute_pucts + argmax (mcts.py:282-315) for D given states: n [D],
   stats [D][24] (sums[10], counts[10], total, min, max), hist [D][172]
   outcome counts (value v at bin v+171), probs [D][10] f32 -> pucts [D][10]
   f64, choice [D] (formula test hook). */
sn_status sn_puct_score(int64_t num, const int32_t* n, const int32_t* stats, const int32_t* hist, const float* probs,
                        double c_puct, double* pucts, int32_t* choice, void* stream);

#ifdef __cplusplus
}
#endif
#endif

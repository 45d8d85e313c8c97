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

#ifdef __cplusplus
}
#endif
#endif

"""Monte-Carlo search agents (reference: rl_6_nimmt/agents/mcts.py).

`MCSAgent` is a drop-in for the reference's: same constructor, card memory,
`forward(state, legal_actions) -> (card, {"log_prob": ...})` and `learn`.
Its playouts run on the GPU (sn_mcs_decide_exact): the numpy global RNG
state is copied to the device, one wave decodes the n_mc playouts' draws in
the reference's exact order (64 stream words per instruction) and plays them
in its lanes, and the advanced state is copied back -- so a seeded
GameSession makes the same choices as the reference.

Deviation: where a legal move received no playout the
reference raises IndexError from a debug f-string (mcts.py:167-170); this
agent returns the best sampled move and logs a warning instead.
"""
import logging
import math

import numpy as np
import torch

from .. import _native as nat
from .base import Agent

logger = logging.getLogger(__name__)

ROWS, THRESHOLD, HAND = 4, 6, 10


class BaseMCAgent(Agent):
    def __init__(self, handsize=10, num_rows=4, num_cards=104, threshold=6, mc_per_card=10, mc_max=100,
                 include_summaries=True, *args, **kwargs):
        super().__init__(*args, **kwargs)
        self.num_players = None
        self.handsize = handsize
        self.num_rows = num_rows
        self.num_cards = num_cards
        self.threshold = threshold
        self.mc_per_card = mc_per_card
        self.mc_max = mc_max
        self.include_summaries = include_summaries
        self.available_cards = []

    # ---------------------------------------------------------- card memory (mcts.py:43-89)
    def forward(self, state, legal_actions, *args, **kwargs):
        n = len(legal_actions)
        if n == self.handsize:
            self._initialize_game(state)
        self._memorize_cards(state, legal_actions)
        if n == 1:
            return legal_actions[0], {"log_prob": torch.tensor(0.0).to(self.device, self.dtype)}
        return self._mcts(legal_actions, state)

    def learn(self, state, reward, action, done, next_state, next_reward, episode_end, num_episode, legal_actions,
              *args, **kwargs):
        raise NotImplementedError

    def _initialize_game(self, state):
        self.available_cards = list(range(self.num_cards))
        self.num_players = int(state[10])

    def _memorize_cards(self, state, legal_actions):
        seen = set(int(c) for c in legal_actions) | set(self._board_from_state(state, flatten=True))
        self.available_cards = [c for c in self.available_cards if c not in seen]

    def _board_from_state(self, state, flatten=True):
        if hasattr(state, "detach"):
            state = state.detach().cpu().numpy()
        cells = np.asarray(state[-self.num_rows * self.threshold:], dtype=np.float64).reshape(self.num_rows, self.threshold)
        rows = [[int(v) for v in row if v >= 0.0] for row in cells]
        return [c for row in rows for c in row] if flatten else rows

    def _compute_n_mc(self, n_actions):
        return min(self.mc_max, self.mc_per_card * math.factorial(n_actions))

    def _mcts(self, legal_actions, state):
        raise NotImplementedError


class MCSAgent(BaseMCAgent):
    """Monte-Carlo search with uniformly random playouts for every seat."""

    def learn(self, *args, **kwargs):
        pass

    def _mcts(self, legal_actions, state):
        nat.require_gpu()
        dev = torch.device("cuda", torch.cuda.current_device())
        board = np.full((1, ROWS, THRESHOLD), -1, dtype=np.int8)
        for r, row in enumerate(self._board_from_state(state, flatten=False)):
            board[0, r, : len(row)] = row
        hand = np.full((1, HAND), -1, dtype=np.int8)
        hand[0, : len(legal_actions)] = sorted(int(c) for c in legal_actions)
        words = np.zeros(4, dtype=np.uint64)
        for c in self.available_cards:
            words[c >> 5] |= np.uint64(1) << np.uint64(c & 31)
        st = np.random.get_state()
        t = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a)).to(dev, dt)
        d_board, d_hand = t(board, torch.int8), t(hand, torch.int8)
        d_avail = t(words.astype(np.uint32).view(np.int32).reshape(1, 4), torch.int32)
        d_key = t(st[1].astype(np.uint32).view(np.int32).reshape(1, 624), torch.int32)
        d_pos = t(np.array([st[2]], dtype=np.int32), torch.int32)
        d_act = torch.zeros(1, dtype=torch.int32, device=dev)
        d_sums = torch.zeros((1, 10), dtype=torch.int32, device=dev)
        d_cnts = torch.zeros((1, 10), dtype=torch.int32, device=dev)
        nat.check(nat.lib().sn_mcs_decide_exact(dev.index, 1, int(self.num_players), nat.ptr(d_board), nat.ptr(d_hand),
                                                nat.ptr(d_avail), int(self.mc_per_card), int(self.mc_max),
                                                nat.ptr(d_key), nat.ptr(d_pos), nat.ptr(d_act), nat.ptr(d_sums),
                                                nat.ptr(d_cnts), nat.stream_handle(dev)), "sn_mcs_decide_exact")
        key = d_key.cpu().numpy().view(np.uint32)[0].copy()
        np.random.set_state((st[0], key, int(d_pos.item()), st[3], st[4]))
        act = int(d_act.item())
        if act < 0:
            act = -act - 2
            logger.warning("MCS: a legal move got no playout (the reference raises IndexError here, quirk Q6)")
        self.last_search = {"sums": d_sums.cpu().numpy()[0], "counts": d_cnts.cpu().numpy()[0]}
        return act, {"log_prob": torch.tensor(0.0).to(self.device, self.dtype)}


# ---------------------------------------------------------------------------
# policy-guided search ("Alpha0.5"): mcts.py:191-323
# ---------------------------------------------------------------------------
from torch import nn  # noqa: E402
from torch.distributions import Categorical  # noqa: E402

from ..utils.nets import MultiHeadedMLP  # noqa: E402
from ..utils.preprocessing import SechsNimmtStateNormalization  # noqa: E402


class PolicyMCSAgent(BaseMCAgent):
    """Monte-Carlo search whose playouts sample every move from a learnable
    policy (mcts.py:191-261).  The search runs on the GPU (sechs_puct.hip:
    candidate rows -> policy MLP via PyTorch-ROCm -> select/step kernels);
    its random numbers are Philox, not numpy/torch's global generators, so
    runs are statistically -- not bitwise -- equivalent to the reference."""

    _puct_root = False

    def __init__(self, hidden_sizes=(100, 100), activation=nn.ReLU(), r_factor=0.1, **kwargs):
        super().__init__(**kwargs)
        self.r_factor = r_factor
        self.preprocessor = SechsNimmtStateNormalization(action=True)
        self.actor = MultiHeadedMLP(self.state_length + 1, hidden_sizes=hidden_sizes, head_sizes=(1,),
                                    activation=activation, head_activations=(None,))
        self.softmax = nn.Softmax(dim=0)
        # the search key is drawn without moving torch's global stream, so
        # seeded constructions init the same weights as the reference's
        rng = torch.random.get_rng_state()
        self.search_seed = int(torch.randint(0, 2**62, (1,)).item())
        torch.random.set_rng_state(rng)
        self._engine = None
        self._decisions = 0

    # policy as in mcts.py:219-228 (host torch; also gives the training log-prob)
    def _compute_policy(self, legal_actions, state):
        state = torch.as_tensor(state).to(self.device, self.dtype).reshape(-1)
        cards = torch.tensor(legal_actions, device=self.device).to(self.dtype)[:, None]
        batch = torch.cat((cards, state[None, :].expand(len(legal_actions), -1)), dim=1)
        (logits,) = self.actor(self.preprocessor(batch))
        return self.softmax(logits).flatten()

    def __getstate__(self):
        # the device search engines (a GPU env handle, captured graphs) are
        # caches: a copy (Tournament.copy_player) builds its own
        d = super().__getstate__() if hasattr(super(), "__getstate__") else dict(self.__dict__)
        d = dict(d)
        d["_engine"] = None
        d.pop("_engines", None)
        return d

    def _search_engine(self):
        from ..puct import BatchedPUCT
        from ..vec_env import VecSechsNimmtEnv

        # one engine per player count (a Tournament seats 2..4): each keeps its
        # captured rollout graphs across games
        engines = self.__dict__.setdefault("_engines", {})
        eng = engines.get(self.num_players)
        if eng is None:
            env = VecSechsNimmtEnv(1, self.num_players, seed=0, rng="philox")
            eng = engines[self.num_players] = BatchedPUCT(
                env, self.actor, mc_per_card=self.mc_per_card, mc_max=self.mc_max, c_puct=getattr(self, "c_puct", 2.0),
                seed=self.search_seed, seats_mask=1, puct_root=self._puct_root, net_dtype=torch.float32, graph=True)
            eng.graph_after = 1  # a shape's second decision captures it
        self._engine = eng
        eng.mc_per_card, eng.mc_max = self.mc_per_card, self.mc_max
        eng.c_puct = float(getattr(self, "c_puct", 2.0))
        return eng

    def _mcts(self, legal_actions, state):
        nat.require_gpu()
        eng = self._search_engine()
        n = len(legal_actions)
        legal = sorted(int(c) for c in legal_actions)
        board = self._board_from_state(state, flatten=False)
        # the other seats' hands are never read by the search (their cards are
        # dealt from the memory); reset_to only needs n distinct cards each
        used = set(legal) | {c for row in board for c in row}
        spare = [c for c in self.available_cards if c not in used] + [c for c in range(104) if c not in used]
        spare = list(dict.fromkeys(spare))
        hands = [legal] + [sorted(spare[i * n:(i + 1) * n]) for i in range(self.num_players - 1)]
        b = np.full((1, ROWS, THRESHOLD), -1, dtype=np.int8)
        for r, row in enumerate(board):
            b[0, r, : len(row)] = row
        h = np.full((1, self.num_players, HAND), -1, dtype=np.int8)
        for p, hand in enumerate(hands):
            h[0, p, : len(hand)] = hand
        eng.env.reset_to(torch.from_numpy(b), torch.from_numpy(h))
        words = np.zeros(4, dtype=np.uint64)
        for c in self.available_cards:
            words[c >> 5] |= np.uint64(1) << np.uint64(c & 31)
        eng.avail.zero_()
        eng.avail[:, 0] = torch.from_numpy(words.astype(np.uint32).view(np.int32)).to(eng.avail.device)
        eng.step_id = self._decisions
        self._decisions += 1
        eng.decide(n, memorize=False)
        best = int(eng.best_index[0].item())
        probs = self._compute_policy(legal, state)
        return legal[best], {"log_prob": torch.log(probs[best])}

    # learning (mcts.py:230-261)
    def learn(self, state, reward, action, done, next_state, next_reward, episode_end, num_episode, legal_actions,
              *args, **kwargs):
        self.history.store(log_prob=kwargs["log_prob"], reward=reward * self.r_factor)
        if not episode_end or not self.training:
            return 0.0
        loss = self._train()
        self.history.clear()
        return loss

    def _train(self):
        log_probs = torch.stack(self.history.rollout()["log_prob"], dim=0)
        loss = -torch.sum(log_probs)
        self._gradient_step(loss)
        return loss.item()

    def _gradient_step(self, loss):
        self.optimizer.zero_grad()
        loss.backward()
        self.optimizer.step()


class PUCTAgent(PolicyMCSAgent):
    """PolicyMCSAgent whose root move is chosen by PUCT (mcts.py:264-323)."""

    _puct_root = True

    def __init__(self, c_puct=2.0, temperature=None, **kwargs):
        super().__init__(**kwargs)
        self.c_puct = c_puct
        self.temperature = temperature

    def _mcts(self, legal_actions, state):
        if self.temperature is not None and self.temperature > 1.0e-12:
            raise NotImplementedError  # mcts.py:318-323 (quirk Q9)
        return super()._mcts(legal_actions, state)

    # host forms of the root formulas (mcts.py:295-315), kept for the API
    def _compute_pucts(self, legal_actions, outcomes, probs):
        n = np.array([len(outcomes[a]) for a in legal_actions])
        hi, lo, mid = self._normalize_q(outcomes)
        q = np.array([np.mean(outcomes[a]) if outcomes[a] else mid for a in legal_actions])
        with np.errstate(invalid="ignore", divide="ignore"):
            q = np.clip((q - lo) / (hi - lo), 0.0, 1.0)
        p = probs.detach().cpu().numpy() if hasattr(probs, "detach") else np.asarray(probs, dtype=np.float32)
        return q + self.c_puct * p * (n.sum() + 1.0e-9) ** 0.5 / (1.0 + n)

    def _normalize_q(self, outcomes):
        every = [o for lst in outcomes.values() for o in lst]
        if len(every) < 10:
            return 0.0, -10.0, -5.0  # quirk Q8: the "mean" is a median, with this fallback
        return np.max(every), np.min(every), np.median(every)


class PUCTCustomedAgent(PUCTAgent):
    """PUCTAgent with a 2-head net (policy logit, value) and no rollouts
    (mcts.py:325-451): every move -- the root included, since the reference
    calls _choose_action_mc with opponent=True (mcts.py:372-374) -- is the
    first argmax of the value head over the legal cards; info carries
    log pi(move) from the policy head and the chosen value as "outcome".
    The reference draws a random environment first (_draw_env) whose other
    hands it never reads; the same numpy shuffle is made here so the global
    stream stays in step with the reference's.  The net is evaluated on the
    host (the agent's device); the batched form is puct.BatchedPUCTCustomed
    (sn_puct_root_rows -> MLP -> sn_pcv_choose on the GPU)."""

    def __init__(self, hidden_sizes=(100, 100), activation=nn.ReLU(), **kwargs):
        super().__init__(hidden_sizes=hidden_sizes, activation=activation, **kwargs)
        self.actor = MultiHeadedMLP(self.state_length + 1, hidden_sizes=hidden_sizes, head_sizes=(2,),
                                    activation=activation, head_activations=(None,))
        self.MSELoss = nn.MSELoss()

    def forward(self, state, legal_actions, *args, **kwargs):
        n = len(legal_actions)
        if n == self.handsize:
            self._initialize_game(state)
        self._memorize_cards(state, legal_actions)
        action, info = self._mcts(legal_actions, state)
        if n == 1:  # mcts.py:347-349
            return legal_actions[0], {"log_prob": torch.tensor(0.0).to(self.device, self.dtype), "outcome": info["outcome"]}
        return action, info

    def _mcts(self, legal_actions, state):
        cards = list(self.available_cards)
        np.random.shuffle(cards)  # _draw_env -> _deal_hands (mcts.py:116-127): only its draws matter
        probs, values = self._compute_policy_and_value(legal_actions, state)
        action_id = torch.argmax(values)
        log_prob = Categorical(probs).log_prob(action_id)
        return int(legal_actions[action_id]), {"log_prob": log_prob, "outcome": values[action_id]}

    def _compute_policy_and_value(self, legal_actions, state):
        state = torch.as_tensor(state).to(self.device, self.dtype).reshape(-1)
        cards = torch.tensor(legal_actions, device=self.device).to(self.dtype)[:, None]
        batch = torch.cat((cards, state[None, :].expand(len(legal_actions), -1)), dim=1)
        (out,) = self.actor(self.preprocessor(batch))
        return self.softmax(out[:, 0]).flatten(), out[:, 1].flatten()

    def learn(self, state, reward, action, done, next_state, next_reward, episode_end, num_episode, legal_actions,
              *args, **kwargs):
        self.history.store(log_prob=kwargs["log_prob"], outcome=kwargs["outcome"], reward=reward * self.r_factor)
        if not episode_end or not self.training:
            return 0.0
        loss = self._train()
        self.history.clear()
        return loss

    def _train(self):
        rollout = self.history.rollout()
        log_probs = torch.stack(rollout["log_prob"], dim=0)
        outcome = torch.stack(rollout["outcome"], dim=0)
        reward_sum = sum(rollout["reward"]) / self.r_factor
        outcome_loss = self.MSELoss(outcome, torch.full(outcome.shape, fill_value=reward_sum))
        policy_loss = -torch.sum(log_probs)
        loss = outcome_loss + policy_loss
        logger.info("loss: %s, policy_loss: %s, outcome_loss: %s", loss.item(), policy_loss.item(), outcome_loss.item())
        self._gradient_step(loss)
        return loss.item()

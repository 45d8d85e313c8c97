"""Episode memories of the learning agents.

`History` is what the PUCT / REINFORCE agents use of the reference's
utils/replay_buffer.py `History` (store / rollout / clear: agents/mcts.py:232,
241,247, agents/policy.py:174-196): an append-only list.

`SequentialHistory` is the ACER agent's replay (replay_buffer.py:206-302): a
ring of whole sequences with the reference's indexing, which the off-policy
replay depends on --
  * capacity `max_length` slots written round-robin; `len` is the number of
    filled slots (the pointer while filling, `max_length` once wrapped);
  * `len` drops back to the pointer at the first push after a wrap, so
    `sample(n)` (Python's global `random.sample` over `range(len)`,
    replay_buffer.py:233-238) never sees the older sequences still held in
    slots >= pointer -- kept, the off-policy replay inherits it;
  * `rollout(n)` returns slots `[len - n, len)` (replay_buffer.py:240-244):
    for n = 1 always the newest sequence;
  * a sequence is built with `store(**step)` (a `first` flag is added per
    step) and pushed with `flush()` (replay_buffer.py:281-302).
"""
import random


class History:
    def __init__(self, max_length=None, dtype=None, device=None):
        self.max_length = max_length
        self.dtype, self.device = dtype, device
        self._items = []

    def store(self, **kwargs):
        self._items.append(kwargs)
        if self.max_length is not None and len(self._items) > self.max_length:
            self._items.pop(0)

    def rollout(self, n=None):
        items = self._items if n is None else self._items[-n:]
        keys = items[0].keys() if items else []
        return {k: [it[k] for it in items] for k in keys}

    def clear(self):
        self._items = []

    def __len__(self):
        return len(self._items)


class SequentialHistory:
    def __init__(self, max_length=None, dtype=None, device=None):
        self.max_length = max_length
        self.dtype, self.device = dtype, device
        self.clear()

    # ------------------------------------------------------------ long-term ring of sequences
    def clear(self):
        self._slots = [None] * (self.max_length or 0)
        self._next = 0
        self._wrapped = False
        self.current_sequence = {}

    def __len__(self):
        if self.max_length is None:
            return self._next
        return self.max_length if self._wrapped else self._next

    def _push(self, seq):
        if self.max_length is None:
            self._slots.append(seq)
            self._next += 1
            return
        self._slots[self._next] = seq
        self._next += 1
        self._wrapped = False
        if self._next >= self.max_length:
            self._next, self._wrapped = 0, True

    @staticmethod
    def _collate(seqs):
        return {k: [s[k] for s in seqs] for k in seqs[0]}

    def rollout(self, n=None):
        m = len(self)
        return self._collate(self._slots[:m] if n is None else self._slots[m - n: m])

    def sample(self, n):
        idx = random.sample(range(len(self)), k=n)
        return idx, None, self._collate([self._slots[i] for i in idx])

    # ------------------------------------------------------------ the sequence being built
    def current_sequence_length(self):
        if not self.current_sequence:
            return 0
        return len(next(iter(self.current_sequence.values())))

    def store(self, **step):
        fresh = self.current_sequence_length() == 0
        if fresh:
            self.current_sequence = {k: [] for k in step}
            self.current_sequence["first"] = []
        for k, v in step.items():
            self.current_sequence[k].append(v)
        self.current_sequence["first"].append(fresh)

    def flush(self):
        assert self.current_sequence_length() > 0
        self._push(self.current_sequence)
        self.current_sequence = {}

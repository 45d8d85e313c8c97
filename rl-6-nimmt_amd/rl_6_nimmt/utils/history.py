"""Episode memory used by the policy agents' `learn` (the reference keeps
it in utils/replay_buffer.py `History`, of which the PUCT agent uses only
store / rollout / clear: agents/mcts.py:232,241,247)."""


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

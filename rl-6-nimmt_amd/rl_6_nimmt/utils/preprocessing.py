"""Observation normalisation for the policy net (reference:
rl_6_nimmt/utils/preprocessing.py:5-57).  Each field of the (action +) 47-int
observation is mapped affinely to about [-1, 1]:
  action, hand, highest card per row, board: (0, cards-1); players: (0, 6);
  cards per row: (1, 5); bull heads per row: (1, 10).
Same float32 operation order as the reference, so outputs match bit for bit
(tests/test_host_cpu.py::test_normalization_golden).  The HIP candidate-row
kernels (sechs_puct.hip) apply the identical arithmetic on the GPU."""
import torch
from torch import nn


class SechsNimmtStateNormalization(nn.Module):
    def __init__(self, cards=104, rows=4, action=False):
        super().__init__()
        self.cards = cards
        self.rows = rows
        self.action = action

    def _fields(self):
        c, r = self.cards - 1, self.rows
        spec = [(1, 0, c)] if self.action else []
        spec += [(10, 0, c), (1, 0, 6), (r, 1, 5), (r, 0, c), (r, 1, 10), (None, 0, c)]
        return spec

    def forward(self, input):
        squeeze = input.dim() == 1
        x = input.unsqueeze(0) if squeeze else input
        parts, pos = [], 0
        for width, lo, hi in self._fields():
            end = x.shape[1] if width is None else pos + width
            parts.append(self._normalize(x[:, pos:end], lo, hi))
            pos = end
        out = torch.cat(parts, dim=1)
        return out.squeeze() if squeeze else out

    @staticmethod
    def _normalize(input, min_, max_, out_min=-1.0, out_max=1.0):
        return out_min + (out_max - out_min) * (input - min_) / (max_ - min_)

"""Training forward of the engines' MLPs with split-K weight gradients.

The fp32 training passes (ACER updates, the PUCT / PUCTCustomed / REINFORCE
episode losses) run the reference's MultiHeadedMLP over 10^5-10^7 candidate
rows at once.  hipBLASLt computes a weight gradient dW = dY^T X with K = rows
on a handful of 32 x 32 output tiles (15.6 ms for 100 x 100 at 26 M rows on
MI355X, tools/acer_profile.py); SplitKLinear computes it as batched partial
products over row chunks + a sum.  The outputs are the module's; the
gradients equal it to the summation order (test_acer_cpu.py).
"""
import os

import torch
from torch import nn


def splitk_wgrad(dy, x, chunks=256):
    """dW = dy^T x over R rows as `chunks` batched GEMMs of R / chunks rows
    each, then a sum: hipBLASLt runs the single [out, R] x [R, in] GEMM of a
    26 M-row ACER batch on a handful of workgroups (15.6 ms for 100 x 100;
    17 ms for a 1-output head) -- the batch of partial products fills the GPU"""
    R = dy.shape[0]
    m = R // chunks
    if m < 1024:
        return dy.t().mm(x)
    main = chunks * m
    w = torch.bmm(dy[:main].view(chunks, m, -1).transpose(1, 2), x[:main].view(chunks, m, -1)).sum(0)
    if main < R:
        w = w + dy[main:].t().mm(x[main:])
    return w


class SplitKLinear(torch.autograd.Function):
    """y = x W^T + b with the weight gradient of splitk_wgrad (the ACER update's
    fp32 training forward over tens of millions of candidate rows)"""

    @staticmethod
    def forward(ctx, x, w, b):
        ctx.save_for_backward(x, w)
        return torch.addmm(b, x, w.t())

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        dx = dy.mm(w) if ctx.needs_input_grad[0] else None
        dw = splitk_wgrad(dy, x) if ctx.needs_input_grad[1] else None
        db = dy.sum(0) if ctx.needs_input_grad[2] else None
        return dx, dw, db


def train_forward(actor, rows):
    """the actor's forward (MultiHeadedMLP: Linear/ReLU latent layers, one
    Linear per head) with SplitKLinear layers; other layouts: actor(rows)"""
    lat = list(actor.latent_net)
    heads = list(actor.head_nets)
    ok = len(lat) % 2 == 0 and all(isinstance(m, nn.Linear) for m in lat[0::2]) and \
        all(isinstance(m, nn.ReLU) for m in lat[1::2]) and \
        all(len(h) == 1 and isinstance(h[0], nn.Linear) for h in heads)
    if not ok or os.environ.get("SECHS_ACER_SPLITK", "1") == "0":
        return actor(rows)
    h = rows
    for lin in lat[0::2]:
        h = torch.relu(SplitKLinear.apply(h, lin.weight, lin.bias))
    return [SplitKLinear.apply(h, hd[0].weight, hd[0].bias) for hd in heads]



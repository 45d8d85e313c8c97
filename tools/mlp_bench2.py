"""Config-4 policy MLP (48-100-100-1, bf16) on one rollout step's rows:
per-layer time for BLAS backends, TunableOp, chunking and the layer-1 split
(obs part once per seat + the card column broadcast-added)."""
import json
import sys
import time

import torch

torch.manual_seed(0)
dev = "cuda"
S, m = 32768 * 4, 5  # seats of 8192 4-player games (every seat deciding), candidates per seat
R = S * m
bf = torch.bfloat16
x = torch.randn(R, 48, device=dev).to(bf)
W1 = (torch.randn(100, 48, device=dev) * 0.1).to(bf)
b1 = (torch.randn(100, device=dev) * 0.1).to(bf)
W2 = (torch.randn(100, 100, device=dev) * 0.1).to(bf)
b2 = (torch.randn(100, device=dev) * 0.1).to(bf)
W3p = torch.zeros(16, 100, device=dev, dtype=bf)
W3p[0] = (torch.randn(100, device=dev) * 0.1).to(bf)
b3p = torch.zeros(16, device=dev, dtype=bf)
res = {}


def timeit(name, f, reps=20):
    for _ in range(3):
        o = f()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        o = f()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t) / reps
    res[name] = round(dt * 1e6, 1)
    print(f"{name:28s} {dt * 1e6:8.1f} us", flush=True)
    return o


h1 = torch._addmm_activation(b1, x, W1.t())
h2 = torch._addmm_activation(b2, h1, W2.t())


def layers(tag):
    timeit(tag + " L1 (K=48)", lambda: torch._addmm_activation(b1, x, W1.t()))
    timeit(tag + " L2 (K=100)", lambda: torch._addmm_activation(b2, h1, W2.t()))
    timeit(tag + " head (N=16)", lambda: torch.addmm(b3p, h2, W3p.t()))
    timeit(tag + " mlp", lambda: torch.addmm(b3p, torch._addmm_activation(b2, torch._addmm_activation(b1, x, W1.t()), W2.t()), W3p.t()))


layers("default")
W1t, W2t, W3t = W1.t().contiguous(), W2.t().contiguous(), W3p.t().contiguous()
timeit("default L2 W^T contiguous", lambda: torch._addmm_activation(b2, h1, W2t))
for lib in ("cublas", "cublaslt", "ck"):
    try:
        torch.backends.cuda.preferred_blas_library(lib)
        layers(lib)
    except Exception as e:  # noqa: BLE001
        print(lib, "unavailable:", str(e)[:120])
torch.backends.cuda.preferred_blas_library("cublaslt")
# chunked: 4 chunks, intermediates of a chunk stay in the MALL
C = 4


def chunked():
    outs = []
    for xc in x.chunk(C):
        outs.append(torch.addmm(b3p, torch._addmm_activation(b2, torch._addmm_activation(b1, xc, W1.t()), W2.t()), W3p.t()))
    return outs


timeit("chunked x4 mlp", chunked)
# layer-1 split in torch ops: base per seat, card column broadcast
xs = x.view(S, m, 48)[:, 0, :].clone()
xs[:, 0] = 0
card = x.view(S, m, 48)[:, :, 0].contiguous()
w1c = W1[:, 0].contiguous()


def split_torch():
    base = torch.addmm(b1, xs, W1.t())
    return torch.relu(torch.addcmul(base[:, None, :], card[:, :, None], w1c[None, None, :])).view(R, 100)


timeit("split L1 torch ops", split_torch)
timeit("split base GEMM only", lambda: torch.addmm(b1, xs, W1.t()))
try:
    import torch.cuda.tunable as tun

    tun.enable(True)
    tun.tuning_enable(True)
    tun.set_max_tuning_duration(30)
    tun.set_filename("/tmp/tunableop_results.csv")
    layers("tunable (tuning)")
    tun.tuning_enable(False)
    layers("tunable")
except Exception as e:  # noqa: BLE001
    print("tunableop unavailable:", str(e)[:200])
print("JSON", json.dumps(res))

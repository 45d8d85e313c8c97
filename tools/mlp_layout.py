"""Layer-2 / head GEMM of the config-4 policy MLP in row-major [R, 100]
(current) vs feature-major [100, R] activations (h^T = W h^T), bf16."""
import time

import torch

torch.manual_seed(0)
dev, bf = "cuda", torch.bfloat16
R = 32768 * 4 * 5
h1 = torch.randn(R, 100, device=dev).to(bf)
h1T = h1.t().contiguous()
W2 = (torch.randn(100, 100, device=dev) * 0.1).to(bf)
b2 = (torch.randn(100, device=dev) * 0.1).to(bf)
W3p = torch.zeros(16, 100, device=dev, dtype=bf)
W3p[0] = 0.1
b3p = torch.zeros(16, device=dev, dtype=bf)
b2c = b2[:, None].contiguous()


def t(name, f, reps=20):
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        f()
    torch.cuda.synchronize()
    print(f"{name:40s} {(time.perf_counter() - t0) / reps * 1e6:8.1f} us", flush=True)


t("L2 row-major addmm_act", lambda: torch._addmm_activation(b2, h1, W2.t()))
t("L2 row-major mm", lambda: torch.mm(h1, W2.t()))
t("L2 feature-major mm W h^T", lambda: torch.mm(W2, h1T))
t("L2 feature-major addmm (bias col)", lambda: torch.addmm(b2c, W2, h1T))
t("L2 feature-major addmm + relu_", lambda: torch.addmm(b2c, W2, h1T).relu_())
h2 = torch._addmm_activation(b2, h1, W2.t())
h2T = h2.t().contiguous()
t("head row-major addmm [R,16]", lambda: torch.addmm(b3p, h2, W3p.t()))
t("head feature-major mm W3 h^T [16,R]", lambda: torch.mm(W3p, h2T))
t("head feature-major mv w3 h^T [R]", lambda: torch.mv(h2T.t(), W3p[0]))
t("head feature-major (1,100)x(100,R)", lambda: torch.mm(W3p[:1], h2T))
# augmented feature-major form: bias as an input column against a ones row
KP = 104
h1a = torch.zeros(KP, R, device=dev, dtype=bf)
h1a[:100] = h1T
h1a[100] = 1
W2a = torch.zeros(KP, KP, device=dev, dtype=bf)
W2a[:100, :100] = W2
W2a[:100, 100] = b2
W2a[100, 100] = 1
zR = torch.zeros(R, device=dev, dtype=bf)
t("L2 aug feature-major _addmm_act(zeros[R])", lambda: torch._addmm_activation(zR, W2a, h1a))
t("L2 aug feature-major mm", lambda: torch.mm(W2a, h1a))
t("L2 aug feature-major mm + relu_", lambda: torch.mm(W2a, h1a).relu_())
ref = torch._addmm_activation(b2, h1, W2.t()).float()
got = torch._addmm_activation(zR, W2a, h1a)[:100].t().float()
print("aug max err vs row-major", (got - ref).abs().max().item(), "ones row", torch._addmm_activation(zR, W2a, h1a)[100].float().unique().tolist())
h2a = torch._addmm_activation(zR, W2a, h1a)
W3a = torch.zeros(16, KP, device=dev, dtype=bf)
W3a[0, :100] = 0.1
t("head aug mm [16,KP]x[KP,R]", lambda: torch.mm(W3a, h2a))
t("head aug mm [1,KP]x[KP,R]", lambda: torch.mm(W3a[:1], h2a))

import torch, time
torch.manual_seed(0)
dev='cuda'
R=32768*4*10
x=torch.randn(R,48,device=dev).to(torch.bfloat16)
W1=torch.randn(100,48,device=dev).to(torch.bfloat16); b1=torch.randn(100,device=dev).to(torch.bfloat16)
W2=torch.randn(100,100,device=dev).to(torch.bfloat16); b2=torch.randn(100,device=dev).to(torch.bfloat16)
W3=torch.randn(1,100,device=dev).to(torch.bfloat16); b3=torch.randn(1,device=dev).to(torch.bfloat16)
F=torch.nn.functional
def base():
    h=F.relu(F.linear(x,W1,b1)); h=F.relu(F.linear(h,W2,b2)); return F.linear(h,W3,b3)
def fused():
    h=torch._addmm_activation(b1,x,W1.t()); h=torch._addmm_activation(b2,h,W2.t()); return F.linear(h,W3,b3)
W3p=torch.zeros(16,100,device=dev,dtype=torch.bfloat16); W3p[0]=W3[0]; b3p=torch.zeros(16,device=dev,dtype=torch.bfloat16); b3p[0]=b3[0]
def fused_pad():
    h=torch._addmm_activation(b1,x,W1.t()); h=torch._addmm_activation(b2,h,W2.t()); return torch.addmm(b3p,h,W3p.t())[:, :1]
w3=W3[0]
def fused_mv():
    h=torch._addmm_activation(b1,x,W1.t()); h=torch._addmm_activation(b2,h,W2.t()); return (torch.mv(h,w3)+b3)[:,None]
def fused_sum():
    h=torch._addmm_activation(b1,x,W1.t()); h=torch._addmm_activation(b2,h,W2.t()); return ((h*w3).sum(-1,dtype=torch.float32)+b3.float())[:,None]
ref=base().float()
for name,f in [('base',base),('fused',fused),('fused_pad',fused_pad),('fused_mv',fused_mv),('fused_sum',fused_sum)]:
    for _ in range(3): o=f()
    torch.cuda.synchronize(); t=time.perf_counter()
    for _ in range(20): o=f()
    torch.cuda.synchronize(); dt=(time.perf_counter()-t)/20
    err=(o.float()-ref).abs().max().item()
    print(f"{name:10s} {dt*1e6:8.1f} us  {R*29800/dt/1e12:6.1f} TFLOP/s  maxerr {err:.3g}")

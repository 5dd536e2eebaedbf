import torch, time
dev='cuda'
N,d=50000,128
dA=torch.randn(N,d,device=dev); W1=torch.randn(d,2*d+1,device=dev)
def t(f,n=50):
    f(); torch.cuda.synchronize(); a=torch.cuda.Event(enable_timing=True); b=torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n): f()
    b.record(); torch.cuda.synchronize(); return a.elapsed_time(b)/n*1e3
Wa=W1[:, :d]; Wac=Wa.contiguous(); WaT=Wa.t().contiguous()
print('slice stride257 mm   %.1f us'%t(lambda: dA.mm(Wa)))
print('contiguous mm        %.1f us'%t(lambda: dA.mm(Wac)))
print('via t().contig.t()   %.1f us'%t(lambda: dA.mm(WaT.t())))
x=torch.randn(N,2*d,device=dev); W=torch.randn(d,2*d,device=dev)
print('x @ W.t() (N,256)x(256,128) %.1f us'%t(lambda: x.mm(W.t())))
h=torch.randn(N,d,device=dev); Wcat=torch.randn(2*d,d,device=dev)
print('h @ Wcat.t() (N,128)x(128,256) %.1f us'%t(lambda: h.mm(Wcat.t())))
g=torch.randn(N,d,device=dev); W2=torch.randn(d,d,device=dev)
print('g @ W2 (N,128)x(128,128) %.1f us'%t(lambda: g.mm(W2)))
print('g @ W2.t() %.1f us'%t(lambda: g.mm(W2.t())))
b=torch.randn(d,device=dev)
print('addmm b + g @ W2.t() %.1f us'%t(lambda: torch.addmm(b,g,W2.t())))

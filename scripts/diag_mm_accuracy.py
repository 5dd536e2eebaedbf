import torch
print("allow_tf32", torch.backends.cuda.matmul.allow_tf32, torch.get_float32_matmul_precision())
try:
    print("fp32_precision", torch.backends.cuda.matmul.fp32_precision)
except Exception as e: print(e)
torch.manual_seed(0)
for (m,k,n) in [(5000,257,128),(128,5000,128),(400,128,128),(5000,128,1)]:
    a=torch.randn(m,k,dtype=torch.float64); b=torch.randn(k,n,dtype=torch.float64)
    ref=a@b
    g=(a.float().cuda()@b.float().cuda()).double().cpu()
    c=(a.float()@b.float()).double()
    sc=(a.abs()@b.abs())
    print(m,k,n,"gpu rel",((g-ref).abs()/sc).max().item(),"cpu rel",((c-ref).abs()/sc).max().item())
x=torch.randn(5000,128,dtype=torch.float64)
bn=torch.nn.BatchNorm1d(128).double()
y64=bn(x)
bnf=torch.nn.BatchNorm1d(128).cuda()
yg=bnf(x.float().cuda()).double().cpu()
print("bn gpu err",(yg-y64).abs().max().item())
ln=torch.nn.LayerNorm(128).double(); lnf=torch.nn.LayerNorm(128).cuda()
print("ln gpu err",(lnf(x.float().cuda()).double().cpu()-ln(x)).abs().max().item())

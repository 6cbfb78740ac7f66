import torch, time
dev='cuda'
gy = torch.randn(65536, 256, device=dev); gs = torch.randn(32, 256, 256, device=dev)
ones_n = torch.ones(65536, device=dev); ones_s = torch.ones(1, 32, device=dev)
def t(f, n=50):
    for _ in range(5): f()
    torch.cuda.synchronize(); e0=torch.cuda.Event(enable_timing=True); e1=torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n): f()
    e1.record(); torch.cuda.synchronize(); return e0.elapsed_time(e1)/n*1e3
print("gy.sum(0)        us", t(lambda: gy.sum(0)))
print("mv(gy.t(), ones) us", t(lambda: torch.mv(gy.t(), ones_n)))
print("ones@gy          us", t(lambda: ones_n[None] @ gy))
print("gs.sum(0)        us", t(lambda: gs.sum(0)))
print("ones_s@gs.view   us", t(lambda: ones_s @ gs.view(32, -1)))
x = torch.randn(65536, 256, device=dev)
print("bmm splitK32     us", t(lambda: torch.bmm(gy.reshape(32, 2048, 256).transpose(1, 2), x.reshape(32, 2048, 256))))
print("mm gy.t()@x      us", t(lambda: gy.t() @ x))
print("bmm splitK64     us", t(lambda: torch.bmm(gy.reshape(64, 1024, 256).transpose(1, 2), x.reshape(64, 1024, 256))))
print("bmm splitK128    us", t(lambda: torch.bmm(gy.reshape(128, 512, 256).transpose(1, 2), x.reshape(128, 512, 256))))
print("tanh 64MB        us", t(lambda: torch.tanh(x)))
print("addmm fwd        us", t(lambda: torch.addmm(ones_n[:256], x, gs[0])))

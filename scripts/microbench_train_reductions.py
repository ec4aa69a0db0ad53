import torch, time
dev = torch.device("cuda")
P = 98304
dy = torch.randn(11, P, 512, device=dev)
ones = torch.ones(P, device=dev)
def t(fn, n=20):
    fn(); torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n): fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n * 1e3
ref = dy.sum(1)
print("sum(1)", t(lambda: dy.sum(1)))
print("matmul ones", t(lambda: torch.matmul(ones, dy)), float((torch.matmul(ones, dy) - ref).abs().max()))
print("two-stage 64", t(lambda: dy.view(11, 64, P // 64, 512).sum(2).sum(1)), float((dy.view(11, 64, P // 64, 512).sum(2).sum(1) - ref).abs().max()))
print("two-stage 256", t(lambda: dy.view(11, 256, P // 256, 512).sum(2).sum(1)))
x = torch.randn(P, 512, device=dev); f = torch.randn(P, 64, device=dev)
print("dx.t()@feat[:, :42]", t(lambda: x.t() @ f[:, :42]))
print("bmm split 64", t(lambda: (x.view(64, -1, 512).transpose(1, 2) @ f.view(64, -1, 64)[..., :42]).sum(0)))
print("dx.t()@feat full64", t(lambda: x.t() @ f))
d_o = torch.randn(P, 4, device=dev)
print("d_o.t()@x", t(lambda: d_o.t() @ x))
print("bmm d_o split", t(lambda: (d_o.view(64, -1, 4).transpose(1, 2) @ x.view(64, -1, 512)).sum(0)))

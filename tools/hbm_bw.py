import torch, time
dev = torch.device("cuda:0")
x = torch.randn(2 * 16 * 4096 * 1024, device=dev)  # K+V fp32 = 537 MB
y = torch.empty(x.numel() // 4, device=dev, dtype=torch.float32)  # 134 MB
z = torch.empty_like(x)
def t(fn, n=20):
    fn(); torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
    e0.record()
    for _ in range(n): fn()
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n
ms = t(lambda: z.copy_(x)); print(f"copy 537MB->537MB {ms:.4f} ms  {2*x.numel()*4/ms/1e9:.2f} TB/s")
ms = t(lambda: torch.sum(x)); print(f"sum 537MB {ms:.4f} ms  {x.numel()*4/ms/1e9:.2f} TB/s")
xv = x.view(-1, 4)
ms = t(lambda: torch.amax(xv, dim=1, out=y)); print(f"amax4 537MB->134MB {ms:.4f} ms  {(x.numel()*4+y.numel()*4)/ms/1e9:.2f} TB/s")

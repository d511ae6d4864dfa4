import sys, torch
sys.path.insert(0, '.')
from chronos.ops import gemm
from chronos import ops
ops.load()
torch.set_printoptions(linewidth=200, precision=2)
for (n, k) in [(16, 512), (16, 2048), (64, 4096)]:
    x = torch.ones(1, k, device='cuda', dtype=torch.bfloat16)
    w = torch.zeros(n, k, device='cuda', dtype=torch.bfloat16)
    for r in range(n):
        w[r, :] = 0
        w[r, r] = 1.0   # y[r] should be 1 (if r < k)
        w[r, k - 1] += 2.0 * (r % 3)
    y = gemm._gemv(x, w)
    ref = x.float() @ w.float().t()
    print(n, k, 'y  ', y[0, :16].float().cpu())
    print(n, k, 'ref', ref[0, :16].cpu())
    x = torch.arange(k, device='cuda').float().remainder(7).to(torch.bfloat16).view(1, k)
    w = torch.randn(n, k, device='cuda').to(torch.bfloat16)
    y = gemm._gemv(x, w); ref = x.float() @ w.float().t()
    print('rand err', (y.float() - ref).abs().max().item(), ref.abs().max().item())

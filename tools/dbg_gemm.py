import sys
import torch
sys.path.insert(0, ".")
from pytorchrec_amd import dense as D, _mrec
dev = torch.device("cuda")
for (Bm, N, K) in [(16, 64, 100), (64, 64, 100), (16, 512, 100), (16, 64, 96)]:
    g = torch.Generator().manual_seed(1)
    dy = D._bf16_rows(torch.randn(Bm, N, generator=g).to(torch.bfloat16).to(dev))
    x = torch.zeros(Bm, D._r8(K), dtype=torch.bfloat16, device=dev)
    x[:, :K] = torch.randn(Bm, K, generator=g).to(torch.bfloat16).to(dev)
    x = x[:, :K]
    dW = torch.empty(N, K, device=dev)
    db = torch.empty(N, device=dev)
    D.gemm(dy, _mrec.LAYOUT_COL, x, _mrec.LAYOUT_COL, N, K, Bm, ones_out=db, out=dW)
    ref = dy.float().T @ x.float()
    e = (dW - ref).abs()
    blocks = [(0, 64), (64, 96), (96, K)]
    print((Bm, N, K), [round(float(e[:, a:b].max()), 5) for a, b in blocks if b > a],
          "db", float((db - dy.float().sum(0)).abs().max()), "rows bad", int((e.max(1).values > 1e-3).sum()))

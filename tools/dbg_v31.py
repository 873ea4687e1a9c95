import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'synthetic-audio-detection_amd')]
import torch
from sad.engine import block_conv
DEV = 'cuda:0'
g = torch.Generator().manual_seed(1)
for (N, H, C) in ((1, 16, 256), (3, 32, 256)):
    x = torch.randn(N, H, H, C, generator=g).to(torch.bfloat16).to(DEV)
    w = (torch.randn(C, 9 * C, generator=g) * (2.0 / (9 * C)) ** 0.5).to(torch.bfloat16).to(DEV)
    b = torch.zeros(C, device=DEV)
    o30 = block_conv(x, w, b, 1, 1, relu=False, variant=30).float()
    o31 = block_conv(x, w, b, 1, 1, relu=False, variant=31 + (int(os.environ.get('AB', '0')) << 8)).float()
    for ab in (1,):
        pass
    torch.cuda.synchronize()
    d = (o30 - o31).abs()
    bad = d > 1e-2
    print(N, H, C, 'max diff', d.max().item(), 'bad frac', bad.float().mean().item())
    if bad.any():
        idx = bad.nonzero()
        print(' bad images', idx[:, 0].unique().tolist()[:10])
        print(' bad rows', idx[:, 1].unique().tolist())
        print(' bad cols', idx[:, 2].unique().tolist())
        ch = idx[:, 3].unique()
        print(' bad channels', ch.tolist()[:64], '... n', ch.numel())
        # per row/col counts for image 0
        print(' per (row) counts', [int(bad[0, r].sum()) for r in range(H)])

import sys, torch
sys.path.insert(0, '.')
import torch.nn.functional as F
from multimodal_siamese_cd_amd import hip
hip.load_library()
dev = torch.device('cuda:0')
def nchw(t): return t.permute(0, 3, 1, 2).contiguous()
bad = {}
for variant in (0, 1):
    hip.set_conv_math('x3'); hip.set_wgrad16(variant)
    for (n, h, w, ci, co) in [(2, 4, 32, 64, 64), (3, 6, 16, 128, 192), (1, 32, 64, 64, 128), (2, 16, 16, 512, 512)]:
        g = torch.Generator().manual_seed(5 * variant + ci + co + h)
        x = torch.randn(n, h, w, ci, generator=g); dy = torch.randn(n, h, w, co, generator=g)
        ref = torch.nn.grad.conv2d_weight(nchw(x), (co, ci, 3, 3), nchw(dy), padding=1)
        xd, dyd = x.to(dev), dy.to(dev)
        nb = 0
        for rep in range(30):
            d, nsplit, nbytes = hip.wgrad_plan(hip.nhwc(dyd), hip.nhwc(xd), 1, hip.TAPS_3X3)
            slabs = torch.full((nbytes // 4,), float('nan'), device=dev) if rep % 2 else torch.empty(nbytes // 4, device=dev)
            hip.conv_wgrad(d, slabs)
            dw = torch.empty(co, ci, 3, 3, device=dev)
            hip.wgrad_finalize(slabs, nsplit, co, 9, ci, 0, ci, dw)
            e = ((dw.cpu() - ref).abs().max() / ref.abs().max()).item()
            if not e < 1e-5: nb += 1
        bad[(variant, n, h, w, ci, co)] = nb
        print(variant, (n, h, w, ci, co), 'nsplit', nsplit, 'bad', nb, flush=True)

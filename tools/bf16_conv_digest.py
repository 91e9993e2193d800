"""Digest of bf16-storage 3x3 conv outputs (fwd + dgrad) over five layer shapes, for A/B builds of libscd (SCD_LIB):
identical digests = bit-identical outputs.  Run from the repo root: PYTHONPATH=. SCD_LIB=<lib> python tools/bf16_conv_digest.py"""
import hashlib
import torch
from multimodal_siamese_cd_amd import hip
hip.load_library()
hip.set_conv_math('bf16')
dev = torch.device('cuda:0')
h = hashlib.sha256()
torch.manual_seed(0)
for n, s, ci, co in [(128, 64, 256, 256), (128, 32, 512, 512), (64, 32, 1024, 256), (128, 16, 512, 512), (64, 64, 128, 256), (128, 128, 128, 128), (64, 128, 256, 128)]:
    x = torch.randn(n, s, s, ci, device=dev).to(torch.bfloat16)
    dy = torch.randn(n, s, s, co, device=dev).to(torch.bfloat16)
    w = torch.randn(co, ci, 3, 3, device=dev) * 0.05
    y = torch.empty(n, s, s, co, device=dev, dtype=torch.bfloat16)
    dx = torch.empty(n, s, s, ci, device=dev, dtype=torch.bfloat16)
    hip.conv_igemm(hip.nhwc(x), s, s, 1, hip.TAPS_3X3, hip.pack_conv3x3(w, 0), co, None, hip.nhwc(y))
    hip.conv_igemm(hip.nhwc(dy), s, s, 1, hip.TAPS_3X3, hip.pack_conv3x3(w, 1), ci, None, hip.nhwc(dx))
    torch.cuda.synchronize()
    h.update(y.view(torch.int16).cpu().numpy().tobytes())
    h.update(dx.view(torch.int16).cpu().numpy().tobytes())
    print(n, s, ci, co, float(y.float().abs().mean()), float(dx.float().abs().mean()))
print('digest', h.hexdigest())

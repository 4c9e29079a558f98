"""Time the low-rank DP member (L_DENSE_WGRAD_LR: fc dW over all W*32 gathered rows) alone on one
GPU for W = 1, 2, 4, 8 (Nature-CNN shapes: K 3136, N 512), mean of 200 launches (events)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dist_dqn_amd.ops import _ext  # noqa: E402

ext = _ext.load(required=True)
dev = 'cuda'
F, H = 3136, 512
for W in (1, 2, 4, 8):
    M = 32 * W
    x = torch.rand(M, F, device=dev).to(torch.bfloat16)
    dh = torch.randn(M, H, device=dev).to(torch.bfloat16)
    dw = torch.zeros(F, H, device=dev)
    db = torch.zeros(H, device=dev)
    run = lambda: ext.qnet_wgrad(12, x.data_ptr(), [M, H, F, 0, 0, 0, 0, 0, 0, 0, 0], dh.data_ptr(), H, dw.data_ptr(),
                                 db.data_ptr(), 0, 0, H, H, 64, 64, 128, 1.0, False, mloop=(M + 63) // 64)
    for _ in range(10):
        run()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(200):
        run()
    e1.record()
    torch.cuda.synchronize()
    print('W=%d  M=%3d  %.2f us/launch' % (W, M, e0.elapsed_time(e1) * 1000 / 200))

"""Phase timing of the fused trunk kernel (s_memtime stamps written by thread 0
of every workgroup): input staging, conv1, conv2, conv3 in shader-clock cycles."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from dist_dqn_amd.config import preset
from dist_dqn_amd.models.network import Network

dev = torch.device('cuda', 0)
DTYPE = sys.argv[1] if len(sys.argv) > 1 else 'bf16'          # python scripts/probe_trunk.py [bf16|fp16|fp32]
cfg = preset('nature', 'Pong-v0', '--dtype=%s --seed=0 --backend=hip' % DTYPE)
net = Network.create_network(cfg, (84, 84, 4), 6, device=dev)
ex = net.executor
p, f = ex.packed(net.online.flat), net.online.flat
frames = torch.randint(0, 256, (1000, 84, 84), dtype=torch.uint8, device=dev)
for B, ninst in ((4, 1), (32, 2), (32, 3), (256, 1)):
    ws = ex._workspace(B, dev)
    sl = torch.randint(0, 1000, (B, 4), dtype=torch.int32, device=dev)
    ex.trunk_prof = torch.zeros(ninst * B * 16, dtype=torch.int64, device=dev)
    for _ in range(20):
        ex._fwd_trunk([sl] * ninst, [p] * ninst, [f] * ninst, ws, B, ninst, frames=frames, fc=False)
    torch.cuda.synchronize()
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    st.record()
    for _ in range(50):
        ex._fwd_trunk([sl] * ninst, [p] * ninst, [f] * ninst, ws, B, ninst, frames=frames, fc=False)
    en.record()
    torch.cuda.synchronize()
    t = ex.trunk_prof.view(-1, 16)[:, [0, 1, 2, 6, 8, 9, 10]].double()
    d = (t[:, 1:] - t[:, :-1]).mean(0).tolist()
    names = ['stage', 'conv1', 'conv2', 'c3mma', 'c3park', 'c3fin']
    # per-XCD clocks are not synchronised: workgroup w runs on XCD w % 8 (part 0 only is stamped,
    # linear id b + inst * B); span / start skew are taken within each XCD, then the max
    xcd = torch.arange(t.shape[0], device=t.device) % 8
    span, skew = 0.0, []
    for x in range(8):
        tx = t[xcd == x]
        if tx.shape[0] == 0:
            continue
        span = max(span, float((tx[:, -1] - tx[:, 0].min()).max()))
        skew.append(tx[:, 0] - tx[:, 0].min())
    s0 = torch.cat(skew)
    print('B=%d ninst=%d  trunk %.2f us/call | block cycles %.0f: %s | span %.0f, start offsets p50 %.0f max %.0f'
          % (B, ninst, st.elapsed_time(en) * 1e3 / 50, sum(d), ' '.join('%s %.0f' % kv for kv in zip(names, d)),
             span, float(s0.median()), float(s0.max())))
ex.trunk_prof = None

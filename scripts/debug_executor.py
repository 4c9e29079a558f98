"""Per-tensor comparison of the HIP executor against the torch oracle (diagnostics)."""
import sys

import torch

sys.path.insert(0, '.')
from tests.test_executor_gpu import _setup, _rel  # noqa: E402

for extra in ['', '--dueling --double_dqn --loss=huber']:
    net, oracle, batch = _setup(extra, 32)
    g_hip = torch.zeros_like(net.online.flat)
    g_ref = torch.zeros_like(net.online.flat)
    loss, prio = net.executor.loss_and_grad(net.online.flat, net.target.flat, batch, g_hip)
    loss_r, prio_r = oracle.loss_and_grad(net.online.flat, net.target.flat, batch, g_ref)
    torch.cuda.synchronize()
    print('extra=%r loss %.6f ref %.6f prio rel %.4f' % (extra, float(loss), float(loss_r), _rel(prio, prio_r)))
    for name in net.layout.names:
        o, n = net.layout.offsets[name], net.layout.numel(name)
        a, b = g_hip[o:o + n], g_ref[o:o + n]
        cos = float(torch.nn.functional.cosine_similarity(a, b, dim=0))
        print('  %-22s rel %.4f cos %.5f |ref| %.3e |hip| %.3e' % (name, _rel(a, b), cos, float(b.norm()),
                                                                  float(a.norm())))
    # activations: trunk output of instance 0 vs oracle
    ws = next(iter(net.executor._ws.values()))
    from dist_dqn_amd.models import torch_net
    import torch.nn.functional as F
    arch = net.arch
    p = net.layout.views(net.online.flat)
    h = batch['states'].float() * net.config.input_scale
    h = h.permute(0, 3, 1, 2)
    acts = []
    for c in arch.convs:
        h = F.relu(F.conv2d(h, p[c.name + '/w'].permute(3, 2, 0, 1), p[c.name + '/b'], stride=c.stride))
        acts.append(h.permute(0, 2, 3, 1).reshape(-1))
    for i, key in enumerate(['x1', 'x2', 'x3']):
        print('  act %s rel %.4f' % (key, _rel(ws[key][0].float(), acts[i])))

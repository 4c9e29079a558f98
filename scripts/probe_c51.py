"""Phase timing (s_memtime, block 0) of the C51 training head (Rainbow config)."""
import torch

from dist_dqn_amd.config import preset
from dist_dqn_amd.models.network import Network

dev = torch.device('cuda', 0)
cfg = preset('nature', 'Pong-v0', '--seed=0 --backend=hip --distributional --noisy --dueling --double_dqn')
net = Network.create_network(cfg, (84, 84, 4), 6, device=dev)
ex = net.executor
B = 32
g = torch.Generator(device=dev).manual_seed(0)
batch = {'states': torch.randint(0, 256, (B, 84, 84, 4), dtype=torch.uint8, device=dev, generator=g),
         'next_states': torch.randint(0, 256, (B, 84, 84, 4), dtype=torch.uint8, device=dev, generator=g),
         'actions': torch.randint(0, 6, (B,), dtype=torch.int32, device=dev, generator=g),
         'rewards': torch.randn(B, device=dev, generator=g), 'dones': torch.zeros(B, device=dev),
         'gammas': torch.full((B,), 0.99, device=dev)}
grad = torch.zeros_like(net.online.flat)
ex.head_prof = torch.zeros(32, dtype=torch.int64, device=dev)
for _ in range(10):
    ex.loss_and_grad(net.online.flat, net.target.flat, batch, grad, net.noise, net.noise_target)
torch.cuda.synchronize()
t = ex.head_prof[:9].double()
d = (t[1:] - t[:-1]).tolist()
names = ['logits(sel)', 'softmax+Q(sel)', 'argmax', 'target logits+softmax+proj', 'online logits+CE',
         'dW (MFMA)', 'dH (MFMA)', 'bias grads']
print('C51 head block-0 cycles: total %.0f | ' % sum(d) + ' | '.join('%s %.0f' % kv for kv in zip(names, d)))
tt = ex.head_prof[10:14].double()
print('wave-0 logits tasks (cycles):', (tt[1:] - tt[:-1]).tolist(), 'from kernel start to first task:', float(tt[0] - t[0]))
t3 = ex.head_prof[[4, 14, 15, 16, 5]].double()
print('online phase split (cycles): wait projection %.0f | rows+softmax %.0f | CE %.0f | reduce+loss %.0f'
      % tuple((t3[1:] - t3[:-1]).tolist()))

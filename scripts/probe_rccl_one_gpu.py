"""Probe: can RCCL (torch.distributed backend "nccl") run 2 ranks on ONE GPU? All-reduce, all-gather
and reduce-scatter of a small tensor; rank 0 prints one JSON line. Launch:
    python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 --master-port P \\
        scripts/probe_rccl_one_gpu.py
"""
import json
import os

import torch
import torch.distributed as dist


def main():
    rank, world = int(os.environ['RANK']), int(os.environ['WORLD_SIZE'])
    torch.cuda.set_device(0)
    dist.init_process_group('nccl', rank=rank, world_size=world, device_id=torch.device('cuda', 0))
    x = torch.full((1 << 20,), float(rank + 1), device='cuda')
    dist.all_reduce(x)
    g = [torch.empty(4, device='cuda') for _ in range(world)]
    dist.all_gather(g, torch.full((4,), float(rank), device='cuda'))
    rs = torch.empty(4, device='cuda')
    dist.reduce_scatter(rs, [torch.full((4,), float(rank + 1), device='cuda') for _ in range(world)])
    torch.cuda.synchronize()
    want = world * (world + 1) / 2
    ok = bool((x == want).all()) and all(bool((g[r] == r).all()) for r in range(world)) and bool((rs == want).all())
    if rank == 0:
        print(json.dumps({'backend': dist.get_backend(), 'world': world, 'ok': ok,
                          'nccl_version': '.'.join(map(str, torch.cuda.nccl.version()))}))
    dist.destroy_process_group()


if __name__ == '__main__':
    main()

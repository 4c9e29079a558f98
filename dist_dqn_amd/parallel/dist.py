"""Process-group bootstrap (reference cluster bootstrap C2,
`/root/reference/src/main.py:169-193`).

The reference builds a TF ``ClusterSpec{ps, worker}`` from ``--ps_hosts`` /
``--worker_hosts`` and starts a gRPC server per process; one PS process
holds the parameters. Here every process is a learner rank of one
``torch.distributed`` group:
  * backend ``nccl`` (= RCCL over xGMI on ROCm) for GPU ranks, ``gloo`` for CPU;
  * rank/world come from torchrun's env (RANK, WORLD_SIZE, LOCAL_RANK,
    MASTER_ADDR/PORT) or, for reference command lines, from
    ``--worker_hosts`` (world = #hosts, master = first host) and ``--task_id``;
  * ``--job=ps`` is accepted and exits immediately: no rank is sacrificed to a
    parameter server (the reference used N-1 of N GPUs, `scripts/dqn_multi_gpu.sh:25-36`).
"""
from __future__ import annotations

import dataclasses
import datetime
import os
from typing import Optional

import torch
import torch.distributed as dist


@dataclasses.dataclass
class DistContext:
    rank: int = 0
    world_size: int = 1
    local_rank: int = 0
    device: torch.device = torch.device('cpu')
    backend: str = 'none'
    # control plane: a gloo group over the same ranks (the default group itself when that is
    # gloo). Stop agreement, restored-path/sidecar broadcast and replica fingerprints go here,
    # as CPU tensors, so they never queue behind (or synchronise with) the GPU stream.
    ctrl_group: object = None

    @property
    def is_chief(self) -> bool:
        return self.rank == 0

    def ctrl_allreduce_max(self, value: int) -> int:
        """max over ranks of a host integer (control plane; no GPU involvement)."""
        if not self.enabled:
            return int(value)
        t = torch.tensor([int(value)], dtype=torch.int64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.ctrl_group)
        return int(t)

    def ctrl_broadcast_object(self, obj, src: int = 0):
        """rank ``src``'s picklable ``obj`` on every rank (control plane)."""
        if not self.enabled:
            return obj
        box = [obj]
        dist.broadcast_object_list(box, src=src, group=self.ctrl_group)
        return box[0]

    @property
    def enabled(self) -> bool:
        return self.world_size > 1

    def barrier(self):
        if self.enabled:
            if self.backend == 'nccl':
                dist.barrier(device_ids=[self.device.index])
            else:
                dist.barrier()


def _from_cluster_flags(config):
    hosts = [h for h in (config.worker_hosts or '').split(',') if h]
    if len(hosts) <= 1:
        return None
    host, port = hosts[0].rsplit(':', 1)
    if host == 'localhost':
        host = '127.0.0.1'
    return dict(rank=config.task_id, world=len(hosts), addr=host, port=port, local_rank=config.gpu_id)


def init_distributed(config=None, device: str = 'auto', timeout_s: int = 600) -> DistContext:
    env_world = int(os.environ.get('WORLD_SIZE', '1'))
    cl = _from_cluster_flags(config) if config is not None and env_world == 1 else None
    if env_world > 1:
        rank, world = int(os.environ['RANK']), env_world
        local_rank = int(os.environ.get('LOCAL_RANK', rank))
    elif cl is not None:
        rank, world, local_rank = cl['rank'], cl['world'], cl['local_rank']
        os.environ.setdefault('MASTER_ADDR', cl['addr'])
        os.environ.setdefault('MASTER_PORT', cl['port'])
    else:
        rank, world, local_rank = 0, 1, int(getattr(config, 'gpu_id', 0) or 0) if config else 0
    if device == 'auto':
        device = getattr(config, 'device', 'auto') if config is not None else 'auto'
    use_gpu = (device in ('auto', 'cuda')) and torch.cuda.is_available()
    if use_gpu:
        ndev = torch.cuda.device_count()
        dev = torch.device('cuda', local_rank % max(ndev, 1))
        torch.cuda.set_device(dev)
    else:
        dev = torch.device('cpu')
    backend = 'none'
    if world > 1:
        backend = 'nccl' if use_gpu else 'gloo'
        # DQN_DIST_BACKEND=gloo: rehearse the multi-rank GPU path with several ranks on ONE
        # device (RCCL refuses two ranks per GPU; gloo stages CUDA tensors through the host)
        backend = os.environ.get('DQN_DIST_BACKEND', backend)
        if not dist.is_initialized():
            kw = dict(backend=backend, rank=rank, world_size=world,
                      timeout=datetime.timedelta(seconds=timeout_s))
            if use_gpu and backend == 'nccl':
                kw['device_id'] = dev
            dist.init_process_group(**kw)
    ctrl = None
    if world > 1 and backend != 'gloo':
        ctrl = dist.new_group(backend='gloo', timeout=datetime.timedelta(seconds=timeout_s))
    return DistContext(rank, world, local_rank, dev, backend, ctrl)


def shutdown(ctx: Optional[DistContext] = None):
    if dist.is_available() and dist.is_initialized():
        try:
            dist.destroy_process_group()
        except Exception:
            pass

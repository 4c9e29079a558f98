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
    # a one-rank process group that still takes every data-parallel code path (the W = 1 probe of
    # the DP step: bench.py --dp_path, tests): collectives over one rank are the identity
    force_dp: bool = False

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

    def ctrl_all_gather_object(self, obj) -> list:
        """[rank 0's obj, rank 1's obj, ...] on every rank (control plane)."""
        if not self.enabled:
            return [obj]
        out = [None] * self.world_size
        dist.all_gather_object(out, obj, group=self.ctrl_group)
        return out

    def device_ids(self) -> list:
        """Every rank's physical device id (`device_id`), gathered over the control plane (cached)."""
        ids = self.__dict__.get('_device_ids')
        if ids is None:
            ids = self.ctrl_all_gather_object(device_id(self.device))
            self.__dict__['_device_ids'] = ids
        return ids

    def ranks_share_gpu(self) -> bool:
        """True when two or more ranks drive the same physical GPU (the one-GPU rehearsals). Decided
        from the gathered PCI ids, so every rank computes the same answer whatever its visible device
        set (``HIP_VISIBLE_DEVICES`` per rank gives device_count() == 1 on every rank of a real node)."""
        if not self.enabled or self.device.type != 'cuda':
            return False
        ids = self.device_ids()
        return len(set(ids)) < len(ids)

    @property
    def enabled(self) -> bool:
        return self.world_size > 1 or self.force_dp

    def barrier(self):
        if self.enabled:
            if self.backend == 'nccl':
                dist.barrier(device_ids=[self.device.index])
            else:
                dist.barrier()


def device_id(dev: torch.device) -> str:
    """Physical identity of a device: 'pci:<domain>:<bus>:<device>' (plus the uuid when the
    runtime reports one) for a GPU, 'cpu' otherwise."""
    if dev.type != 'cuda':
        return 'cpu'
    p = torch.cuda.get_device_properties(dev)
    pci = 'pci:%04x:%02x:%02x' % (getattr(p, 'pci_domain_id', 0), getattr(p, 'pci_bus_id', 0),
                                  getattr(p, 'pci_device_id', 0))
    uuid = str(getattr(p, 'uuid', '') or '')
    return pci + ('/' + uuid if uuid else '')


def _from_cluster_flags(config):
    hosts = [h for h in (config.worker_hosts or '').split(',') if h]
    if len(hosts) <= 1:
        return None
    host, port = hosts[0].rsplit(':', 1)
    if host == 'localhost':
        host = '127.0.0.1'
    return dict(rank=config.task_id, world=len(hosts), addr=host, port=port, local_rank=config.gpu_id)


def init_distributed(config=None, device: str = 'auto', timeout_s: int = 600, force_dp: bool = False) -> DistContext:
    """``force_dp`` (one process only): form a one-rank process group anyway and report the context
    enabled, so the data-parallel step runs at W = 1 (its collectives are the identity)."""
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
    backend = 'none'
    force_dp = bool(force_dp) and world == 1
    if force_dp:
        os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
        if 'MASTER_PORT' not in os.environ:
            import socket
            with socket.socket() as sk:
                sk.bind(('127.0.0.1', 0))
                os.environ['MASTER_PORT'] = str(sk.getsockname()[1])
    if world > 1 or force_dp:
        backend = 'nccl' if use_gpu else 'gloo'
        # DQN_DIST_BACKEND=gloo: rehearse the multi-rank GPU path with several ranks on ONE
        # device (RCCL refuses two ranks per GPU; gloo stages CUDA tensors through the host)
        backend = os.environ.get('DQN_DIST_BACKEND', backend)
    if use_gpu:
        ndev = torch.cuda.device_count()
        if ndev == 0:
            raise RuntimeError('rank %d: no visible GPU' % rank)
        # (local_rank % ndev: a rank that sees only its own GPU -- per-rank HIP_VISIBLE_DEVICES, SLURM
        # --gpus-per-task=1, the reference's --gpu_id flags -- has local rank 1..N-1 but one device.
        # Real sharing of one physical GPU is decided after the group exists, from the PCI ids.)
        dev = torch.device('cuda', local_rank % ndev)
        torch.cuda.set_device(dev)
    else:
        dev = torch.device('cpu')
    if (world > 1 or force_dp) and not dist.is_initialized():
        kw = dict(backend=backend, rank=rank, world_size=world, timeout=datetime.timedelta(seconds=timeout_s))
        if use_gpu and backend == 'nccl':
            kw['device_id'] = dev
        dist.init_process_group(**kw)
    ctrl = None
    if (world > 1 or force_dp) and backend != 'gloo':
        ctrl = dist.new_group(backend='gloo', timeout=datetime.timedelta(seconds=timeout_s))
    ctx = DistContext(rank, world, local_rank, dev, backend, ctrl, force_dp)
    if ctx.enabled and use_gpu:
        # gathered HERE, on every rank, and cached: a later ranks_share_gpu() is then never a
        # collective that only some ranks reach (the --async_ps server builds no Learner)
        ctx.device_ids()
    if world > 1 and use_gpu and backend == 'nccl' and ctx.ranks_share_gpu():
        # RCCL needs one GPU per rank: say so here (every rank computes the same answer from the
        # gathered PCI ids) instead of a "Duplicate GPU detected" abort at the first collective
        raise RuntimeError('rank %d (local rank %d, %s): ranks share a physical GPU (%s). Launch at most one '
                           'rank per GPU, or set DQN_DIST_BACKEND=gloo to rehearse several ranks on one GPU.'
                           % (rank, local_rank, device_id(dev), ctx.device_ids()))
    if ctx.enabled:
        first_contact(ctx)
    return ctx


def first_contact(ctx: DistContext):
    """The first collective on the data backend: a 4-element SUM of rank-stamped values on the
    rank's own device, checked exactly. It runs right after the process group forms and BEFORE any
    xgmi / IPC setup, so a broken RCCL install, a duplicate device or a wrong topology fails
    here with its own message instead of inside the transport probe or the first SGD step."""
    W = ctx.world_size
    t = torch.tensor([1.0, float(ctx.rank), float(ctx.rank * ctx.rank), 3.0], device=ctx.device)
    try:
        dist.all_reduce(t)
        got = t.cpu().tolist()
    except Exception as e:  # noqa: BLE001
        raise RuntimeError('first %s collective failed on rank %d of %d (device %s, %s): %s'
                           % (ctx.backend, ctx.rank, W, ctx.device, device_id(ctx.device), e)) from e
    want = [float(W), W * (W - 1) / 2.0, (W - 1) * W * (2 * W - 1) / 6.0, 3.0 * W]
    if got != want:
        raise RuntimeError('first %s collective returned %s on rank %d, expected %s'
                           % (ctx.backend, got, ctx.rank, want))


def shutdown(ctx: Optional[DistContext] = None):
    if dist.is_available() and dist.is_initialized():
        try:
            dist.destroy_process_group()
        except Exception:
            pass

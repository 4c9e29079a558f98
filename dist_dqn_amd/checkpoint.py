"""Checkpoint / resume with the reference's layout.

The reference relies on ``tf.train.Supervisor`` (`/root/reference/src/main.py:136-143`):
every 600 s the chief saves all global variables to
``<logdir>/model.ckpt-<global_step>`` plus a ``checkpoint`` index file, and
``managed_session`` restores the latest one on start.

Kept here:
  * file names: ``<logdir>/checkpoint`` (text index in TF's
    ``model_checkpoint_path: "..."`` format) and ``model.ckpt-<step>``;
  * tensor names and layouts: TF variable names (``conv1/w`` ...), conv HWIO,
    dense [in, out], NHWC flatten order, optimizer slots with TF slot names
    (``conv1/w/RMSProp`` ...), ``global_step``; ``target/*`` only with
    ``--disable_target_replication``.
Storage is safetensors (no pickle; loads execute nothing). Not saved, as in
the reference: replay, epsilon, local training_steps, stats; the agent
re-syncs the target after restore. ``--save_agent_state`` adds an opt-in
JSON sidecar with epsilon and training_steps.
"""
from __future__ import annotations

import contextlib
import glob
import json
import os
import re
import threading
import weakref
import time
from typing import Dict, Optional

import torch
from safetensors.torch import load_file, save_file

_INDEX = 'checkpoint'
_PREFIX = 'model.ckpt'


def _ckpt_path(logdir: str, step: int) -> str:
    return os.path.join(logdir, '%s-%d' % (_PREFIX, step))


def latest_checkpoint(logdir: str) -> Optional[str]:
    idx = os.path.join(logdir, _INDEX)
    if os.path.exists(idx):
        with open(idx) as f:
            for line in f:
                m = re.match(r'model_checkpoint_path:\s*"(.*)"', line.strip())
                if m:
                    p = m.group(1)
                    p = p if os.path.isabs(p) else os.path.join(logdir, p)
                    if os.path.exists(p):
                        return p
    files = sorted(glob.glob(os.path.join(logdir, _PREFIX + '-*')),
                   key=lambda p: int(re.findall(r'-(\d+)$', p)[0]) if re.findall(r'-(\d+)$', p) else -1)
    files = [f for f in files if re.search(r'-\d+$', f)]
    return files[-1] if files else None


def save(logdir: str, tensors: Dict[str, torch.Tensor], step: int, max_to_keep: int = 5,
         sidecar: Optional[dict] = None) -> str:
    os.makedirs(logdir, exist_ok=True)
    path = _ckpt_path(logdir, step)
    tmp = path + '.tmp'
    save_file({k: v.detach().cpu().contiguous() for k, v in tensors.items()}, tmp,
              metadata={'format': 'dist_dqn_amd/tf-layout-v1', 'global_step': str(step)})
    os.replace(tmp, path)
    if sidecar is not None:
        with open(path + '.agent.json', 'w') as f:
            json.dump(sidecar, f)
    kept = sorted(glob.glob(os.path.join(logdir, _PREFIX + '-*')))
    kept = [k for k in kept if re.search(r'-\d+$', k)]
    kept.sort(key=lambda p: int(re.findall(r'-(\d+)$', p)[0]))
    for old in kept[:-max_to_keep] if max_to_keep > 0 else []:
        for f in (old, old + '.agent.json'):
            if os.path.exists(f):
                os.remove(f)
    kept = kept[-max_to_keep:] if max_to_keep > 0 else kept
    with open(os.path.join(logdir, _INDEX + '.tmp'), 'w') as f:
        f.write('model_checkpoint_path: "%s"\n' % os.path.basename(path))
        for k in kept:
            f.write('all_model_checkpoint_paths: "%s"\n' % os.path.basename(k))
    os.replace(os.path.join(logdir, _INDEX + '.tmp'), os.path.join(logdir, _INDEX))
    return path


def load(path: str) -> Dict[str, torch.Tensor]:
    return load_file(path)


def load_sidecar(path: str) -> Optional[dict]:
    p = path + '.agent.json'
    if os.path.exists(p):
        with open(p) as f:
            return json.load(f)
    return None


_MANAGERS: "weakref.WeakSet" = weakref.WeakSet()


def quiesce_writers():
    """Join every live manager's asynchronous checkpoint writer (``Learner`` before a HIP graph
    capture: the writer's D2H copies, event waits and snapshot frees must not interleave with a
    capture on the training thread)."""
    for m in list(_MANAGERS):
        m.join_writer()


class CheckpointManager:
    """Chief-only periodic saver (TF Supervisor's ``save_model_secs`` = 600 by default).

    A periodic save costs the training thread one device-side snapshot (D2D copies on a side
    stream, ``Network.snapshot``); a writer thread does the D2H transfer and the file write.
    Before a save ``check_fn`` (e.g. the xgmi transport's error-word read) must pass: a state
    that may hold a partly reduced gradient is never written. Momentum-0 RMSProp defers its
    never-read ``mom`` slot (``FlatOptimizer.defers_slots``): a due save first asks the next
    step to store it and is written after that step."""

    def __init__(self, logdir: str, network, is_chief: bool = True, save_secs: int = 600,
                 max_to_keep: int = 5, agent_state_fn=None, check_fn=None, async_write: bool = True):
        self.logdir = logdir
        self.network = network
        self.is_chief = is_chief
        self.save_secs = save_secs
        self.max_to_keep = max_to_keep
        self.agent_state_fn = agent_state_fn
        self.check_fn = check_fn
        self.async_write = async_write
        self._last = time.time()
        self._lock = threading.Lock()
        self._armed = False
        self._writer: Optional[threading.Thread] = None
        _MANAGERS.add(self)
        self._write_error: Optional[BaseException] = None
        self.last_path: Optional[str] = None
        # optional context-manager factory held around the snapshot copies when another host
        # thread updates the parameters on its own stream (the native async-PS server: its
        # updates pause, so parameters, slots and global_step come from one update)
        self.quiesce = None

    def restore(self) -> Optional[str]:
        path = latest_checkpoint(self.logdir)
        if path is None:
            return None
        self.network.load_state_dict(load(path))
        return path

    def _opt(self):
        return getattr(self.network, 'optimizer', None)

    def arm_slots(self):
        """Store the optimizer's deferred slots on the following steps (until the next save)."""
        opt = self._opt()
        if self.is_chief and not self._armed and getattr(opt, 'defers_slots', False):
            opt.request_slots(True)
            self._armed = True

    def maybe_save(self, force: bool = False) -> Optional[str]:
        """Save when due (or ``force``: synchronous). Returns the checkpoint path, or None when
        nothing was saved yet or the writer thread is writing it (``wait()`` joins it and returns
        the path)."""
        if not self.is_chief:
            return None
        now = time.time()
        if not force and (self.save_secs <= 0 or now - self._last < self.save_secs):
            return None
        opt = self._opt()
        if not force and not self._armed and getattr(opt, 'defers_slots', False):
            opt.request_slots(True)      # the next step stores the deferred slot; save after it
            self._armed = True
            return None
        if self.check_fn is not None:
            self.check_fn()              # raises: this state is not written
        with self._lock:
            self._last = now
            self.wait()                  # one write in flight at a time
            quiesce = self.quiesce
            with (quiesce() if quiesce is not None else contextlib.nullcontext()):
                snap, ev = self.network.snapshot() if hasattr(self.network, 'snapshot') else (None, None)
                if quiesce is not None and ev is not None:
                    ev.synchronize()     # the copies land before the quiesced writer resumes
            if self._armed:
                opt.request_slots(False)
                self._armed = False
            side = self.agent_state_fn() if self.agent_state_fn else None
            if snap is None:
                sd = self.network.state_dict()
                self.last_path = save(self.logdir, sd, int(sd['global_step']), self.max_to_keep, side)
                return self.last_path
            if not self.async_write or force or ev is None:
                if ev is not None:
                    ev.synchronize()
                sd = self.network.state_dict_from(snap)
                self.last_path = save(self.logdir, sd, int(sd['global_step']), self.max_to_keep, side)
                return self.last_path

            def write():
                try:
                    ev.synchronize()
                    sd = self.network.state_dict_from(snap)
                    self.last_path = save(self.logdir, sd, int(sd['global_step']), self.max_to_keep, side)
                except BaseException as e:  # pragma: no cover - reported by wait()
                    self._write_error = e

            self._writer = threading.Thread(target=write, name='ckpt-writer', daemon=True)
            self._writer.start()
            return None                  # (the path is known once the writer has the step: wait())

    def join_writer(self):
        """Join the writer thread of the last asynchronous save, keeping its error (if any) for the
        next ``wait()``: afterwards no host thread of this manager touches the GPU or frees a
        snapshot buffer (the learner calls this before a graph capture)."""
        w = self._writer
        if w is not None:
            w.join()

    def wait(self) -> Optional[str]:
        """Join the writer thread of the last asynchronous save (re-raising its error)."""
        w, self._writer = self._writer, None
        if w is not None:
            w.join()
        if self._write_error is not None:
            e, self._write_error = self._write_error, None
            raise e
        return self.last_path

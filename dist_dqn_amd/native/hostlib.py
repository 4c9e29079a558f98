"""ctypes bindings of ``dist_dqn_amd/libdqn_host.so`` (csrc/host/*.cpp).

CPU actor processes use these instead of the torch extension: the SPSC
transition rings and the inference mailboxes live in POSIX shared memory and
need real acquire/release atomics across processes, which Python cannot do
itself; the library has no torch or HIP dependency, so an actor process stays
a small numpy process (Ape-X scale: hundreds of them per node).
"""
from __future__ import annotations

import ctypes as C
import os
from typing import Optional

import numpy as np

_PATH = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'libdqn_host.so')
_lib: Optional['HostLib'] = None

_u8p = C.POINTER(C.c_uint8)


def _ptr(a) -> int:
    """Address of a numpy array or an int address."""
    if isinstance(a, np.ndarray):
        return a.ctypes.data
    return int(a)


class HostLib:
    def __init__(self, path: str = _PATH):
        if not os.path.exists(path):
            raise ImportError('%s is missing: run `python setup.py build_ext --inplace`' % path)
        L = C.CDLL(path)
        vp, i64, u64, sz = C.c_void_p, C.c_int64, C.c_uint64, C.c_size_t
        sig = {
            'dqnh_ring_bytes': (sz, [u64, u64]), 'dqnh_ring_init': (None, [vp, u64, u64]),
            'dqnh_ring_push': (i64, [vp, vp, i64]), 'dqnh_ring_pop': (i64, [vp, vp, i64]),
            'dqnh_ring_size': (i64, [vp]),
            'dqnh_mbox_stride': (i64, [i64]), 'dqnh_mbox_region_bytes': (sz, [i64, i64]),
            'dqnh_mbox_init': (None, [vp, i64, i64]), 'dqnh_mbox_set_stop': (None, [vp, i64]),
            'dqnh_mbox_stopped': (i64, [vp]), 'dqnh_mbox_request': (i64, [vp, i64, i64, vp, i64]),
            'dqnh_mbox_collect': (i64, [vp, i64, i64, vp, vp, vp, i64]),
            'dqnh_mbox_respond': (None, [vp, i64, vp, vp, vp, i64]),
            'dqnh_preprocess': (None, [vp, C.c_int, C.c_int, vp, C.c_int, C.c_int]),
            'dqnh_crc32c': (C.c_uint32, [vp, sz]),
            'dqnh_apex_ingest': (None, [vp, i64, vp, C.c_int, C.c_int, C.c_double, i64, vp, vp, i64, vp]),
            'dqnh_apex_ingest_many': (None, [i64, vp, vp, i64, i64, i64, C.c_int, C.c_int, C.c_double, i64, vp, vp,
                                             i64, vp]),
        }
        for name, (res, args) in sig.items():
            f = getattr(L, name)
            f.restype, f.argtypes = res, args
        self.L = L
        self.path = path

    # -------------------------------------------------------------- rings
    def ring_bytes(self, capacity: int, record_bytes: int) -> int:
        return int(self.L.dqnh_ring_bytes(capacity, record_bytes))

    def ring_init(self, buf, capacity: int, record_bytes: int):
        self.L.dqnh_ring_init(_ptr(buf), capacity, record_bytes)

    def ring_push(self, buf, recs: np.ndarray, n: int) -> int:
        return int(self.L.dqnh_ring_push(_ptr(buf), _ptr(recs), n))

    def ring_pop(self, buf, out: np.ndarray, max_n: int) -> int:
        return int(self.L.dqnh_ring_pop(_ptr(buf), _ptr(out), max_n))

    def ring_size(self, buf) -> int:
        return int(self.L.dqnh_ring_size(_ptr(buf)))

    # ---------------------------------------------------------- mailboxes
    def mbox_region_bytes(self, n: int, state_bytes: int) -> int:
        return int(self.L.dqnh_mbox_region_bytes(n, state_bytes))

    def mbox_init(self, region, n: int, state_bytes: int):
        self.L.dqnh_mbox_init(_ptr(region), n, state_bytes)

    def mbox_set_stop(self, region, v: int = 1):
        self.L.dqnh_mbox_set_stop(_ptr(region), v)

    def mbox_stopped(self, region) -> bool:
        return bool(self.L.dqnh_mbox_stopped(_ptr(region)))

    def mbox_request(self, region, i: int, state: np.ndarray, timeout_us: int = -1) -> int:
        """Post `state` in slot i and wait for the server's action (-1 timeout, -2 stop)."""
        return int(self.L.dqnh_mbox_request(_ptr(region), i, state.nbytes, _ptr(state), timeout_us))

    def mbox_collect(self, region, n: int, state_bytes: int, out_states: np.ndarray, out_ids: np.ndarray,
                     out_seq: np.ndarray, max_batch: int) -> int:
        return int(self.L.dqnh_mbox_collect(_ptr(region), n, state_bytes, _ptr(out_states), _ptr(out_ids),
                                            _ptr(out_seq), max_batch))

    def mbox_respond(self, region, state_bytes: int, ids: np.ndarray, seq: np.ndarray, actions: np.ndarray,
                     m: int):
        self.L.dqnh_mbox_respond(_ptr(region), state_bytes, _ptr(ids), _ptr(seq), _ptr(actions), m)

    # ------------------------------------------------------------- images
    def preprocess(self, rgb: np.ndarray, H: int, W: int, out: Optional[np.ndarray] = None) -> np.ndarray:
        """RGB uint8 [Hs, Ws, 3] -> gray + bilinear resize uint8 [H, W] (cv2-compatible fixed point)."""
        rgb = np.ascontiguousarray(rgb, dtype=np.uint8)
        if out is None:
            out = np.empty((H, W), dtype=np.uint8)
        self.L.dqnh_preprocess(_ptr(rgb), rgb.shape[0], rgb.shape[1], _ptr(out), H, W)
        return out

    # ------------------------------------------------------------- Ape-X
    def apex_ingest(self, ring, max_n: int, actor_state: np.ndarray, k: int, nstep: int, gamma: float,
                    frame_bytes: int, stage: np.ndarray, returns: np.ndarray, out: np.ndarray):
        """One actor ring -> replay staging (csrc/host/apex_ingest.cpp). stage: int64[13] in
        DqnIngestStage order (updated in place); out: int64[5] = consumed, frames, episodes,
        returns written, stage full."""
        assert actor_state.dtype == np.int32 and stage.dtype == np.int64 and out.dtype == np.int64
        assert returns.dtype == np.float32
        self.L.dqnh_apex_ingest(_ptr(ring), max_n, _ptr(actor_state), k, nstep, gamma, frame_bytes, _ptr(stage),
                                _ptr(returns), returns.size, _ptr(out))

    def apex_ingest_many(self, rings: np.ndarray, states: np.ndarray, first: int, max_n: int, k: int, nstep: int,
                         gamma: float, frame_bytes: int, stage: np.ndarray, returns: np.ndarray, out: np.ndarray):
        """apex_ingest over every ring (int64 addresses) from actor ``first`` on, in one call;
        out: int64[6] = consumed, frames, episodes, returns written, stage full, resume actor."""
        assert rings.dtype == np.int64 and states.dtype == np.int32 and states.ndim == 2
        assert states.shape[0] == rings.size and out.size >= 6
        self.L.dqnh_apex_ingest_many(rings.size, _ptr(rings), _ptr(states), states.shape[1], first, max_n, k, nstep,
                                     gamma, frame_bytes, _ptr(stage), _ptr(returns), returns.size, _ptr(out))

    def crc32c(self, data: bytes) -> int:
        b = np.frombuffer(data, dtype=np.uint8)
        return int(self.L.dqnh_crc32c(_ptr(b), b.nbytes))


def load() -> HostLib:
    global _lib
    if _lib is None:
        _lib = HostLib()
    return _lib

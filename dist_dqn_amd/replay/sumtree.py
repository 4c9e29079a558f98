"""Device sum-tree / min-tree for prioritized replay (Schaul et al. 2016).

Layout: implicit complete binary tree in one f32 array of 2P entries
(P = next power of two >= capacity; root at 1, leaf i at P + i). The min-tree
(same layout, +inf for empty leaves) gives the exact max importance weight
``(N * p_min / total) ** -beta`` without a reduction pass.

Kernels (`csrc/kernels/sumtree.hip`):
  * sample: B lanes, stratified u_i = (i + U_i) * total / B, each lane descends
    log2(P) levels (reads only: no hazards);
  * update: ONE workgroup writes the B leaves, then recomputes ancestors level
    by level with a barrier between levels — lanes whose paths merge write the
    same value, so duplicate indices in a batch are last-writer-wins on the
    leaf and exact on every parent.
"""
from __future__ import annotations

import torch

from ..ops import kernels


class DeviceSumTree:
    def __init__(self, capacity: int, device):
        P = 1
        while P < capacity:
            P *= 2
        self.P = P
        self.capacity = capacity
        self.device = torch.device(device)
        self.sum = torch.zeros(2 * P, dtype=torch.float32, device=self.device)
        self.min = torch.full((2 * P,), float('inf'), dtype=torch.float32, device=self.device)
        # running max of p^alpha, new transitions enter with it (initial 1.0)
        self.max_p = torch.ones(1, dtype=torch.float32, device=self.device)

    def set_max_priority(self, idx: torch.Tensor):
        kernels.sumtree_set(self, idx, None, 0.0, 0.0, use_max=True)

    def update(self, idx: torch.Tensor, td_abs: torch.Tensor, alpha: float, eps: float):
        kernels.sumtree_set(self, idx, td_abs, alpha, eps, use_max=False)

    def sample(self, rng_state, size_dev, beta, idx_out, w_out):
        kernels.sumtree_sample(self, rng_state, size_dev, beta, idx_out, w_out)

    def total(self) -> float:
        return float(self.sum[1])

"""Architecture specs: one description consumed by BOTH executors
(the torch oracle in `torch_net.py` and the fused HIP executor in
`dist_dqn_amd/ops/executor.py`).

Reference models:
  * ``simple`` — `SimpleNetwork` (`/root/reference/src/network.py:258-313`):
    in -> 20 tanh -> 20 tanh -> A, L2 on all three weights.
  * ``cnn``    — `ConvNetwork` (`/root/reference/src/network.py:317-424`):
    3 x [conv SAME + b, ReLU, maxpool 2x2/2 SAME] -> flatten(HWC) ->
    FC256 ReLU -> A, L2 on the two FC weights.
Extension:
  * ``nature`` — Mnih et al. 2015: VALID convs 32x8x8/4, 64x4x4/2, 64x3x3/1,
    no pooling, FC512 ReLU -> A.
Heads (any network): plain, dueling (V + A - mean A), distributional (C51
atoms), noisy FC layers (factorised Gaussian).

Parameter names are the TF variable names of the reference
(`conv1/w` ..., `output/b`) so the checkpoint layout round-trips; weight
layouts are the TF ones: conv HWIO ``[kh, kw, cin, cout]``, dense ``[in, out]``.
"""
from __future__ import annotations

import dataclasses
import math
from typing import List, Optional, Sequence, Tuple


@dataclasses.dataclass(frozen=True)
class ConvSpec:
    name: str
    k: int
    stride: int
    cin: int
    cout: int
    padding: str          # 'SAME' | 'VALID'
    pool: bool            # 2x2/2 SAME max-pool after ReLU
    in_hw: Tuple[int, int]

    @property
    def conv_hw(self) -> Tuple[int, int]:
        return tuple(_out(n, self.k, self.stride, self.padding) for n in self.in_hw)

    @property
    def out_hw(self) -> Tuple[int, int]:
        h, w = self.conv_hw
        if self.pool:
            return (_out(h, 2, 2, 'SAME'), _out(w, 2, 2, 'SAME'))
        return (h, w)

    def pads(self) -> Tuple[int, int, int, int]:
        """(top, bottom, left, right) TF padding of the convolution."""
        (ih, iw), (oh, ow) = self.in_hw, self.conv_hw
        return _tf_pads(ih, oh, self.k, self.stride, self.padding) + _tf_pads(iw, ow, self.k, self.stride, self.padding)

    def pool_pads(self) -> Tuple[int, int, int, int]:
        (h, w), (oh, ow) = self.conv_hw, self.out_hw
        return _tf_pads(h, oh, 2, 2, 'SAME') + _tf_pads(w, ow, 2, 2, 'SAME')


@dataclasses.dataclass(frozen=True)
class DenseSpec:
    name: str
    fin: int
    fout: int
    act: Optional[str]    # 'relu' | 'tanh' | None
    reg: bool = True      # included in the L2 term
    noisy: bool = False


@dataclasses.dataclass(frozen=True)
class ArchSpec:
    network: str
    input_shape: Tuple[int, ...]      # (H, W, C) for conv nets, (D,) for MLP
    num_actions: int
    convs: Tuple[ConvSpec, ...]
    trunk: Tuple[DenseSpec, ...]      # shared dense layers after the convs
    head: Tuple[DenseSpec, ...]       # plain: Q stream; dueling: advantage stream
    value: Tuple[DenseSpec, ...] = ()  # dueling value stream (empty if not dueling)
    atoms: int = 1
    v_min: float = -10.0
    v_max: float = 10.0
    noisy: bool = False
    noisy_sigma0: float = 0.5

    @property
    def dueling(self) -> bool:
        return len(self.value) > 0

    @property
    def distributional(self) -> bool:
        return self.atoms > 1

    @property
    def is_conv(self) -> bool:
        return len(self.convs) > 0

    @property
    def flat_features(self) -> int:
        if not self.convs:
            return self.input_shape[0]
        c = self.convs[-1]
        return c.out_hw[0] * c.out_hw[1] * c.cout

    def dense_layers(self) -> List[DenseSpec]:
        return list(self.trunk) + list(self.value) + list(self.head)

    def param_specs(self) -> List[Tuple[str, Tuple[int, ...], str]]:
        """Ordered (tf_name, tf_shape, kind) — kind in {w, b, w_sigma, b_sigma}."""
        out = []
        for c in self.convs:
            out.append((c.name + '/w', (c.k, c.k, c.cin, c.cout), 'w'))
            out.append((c.name + '/b', (c.cout,), 'b'))
        for d in self.dense_layers():
            out.append((d.name + '/w', (d.fin, d.fout), 'w'))
            out.append((d.name + '/b', (d.fout,), 'b'))
            if d.noisy:
                out.append((d.name + '/w_sigma', (d.fin, d.fout), 'w_sigma'))
                out.append((d.name + '/b_sigma', (d.fout,), 'b_sigma'))
        return out

    def reg_names(self) -> List[str]:
        return [d.name + '/w' for d in self.dense_layers() if d.reg]

    def num_params(self) -> int:
        return sum(math.prod(s) for _, s, _ in self.param_specs())

    def forward_flops(self) -> int:
        """MACs*2 of one forward pass for one sample."""
        f = 0
        for c in self.convs:
            oh, ow = c.conv_hw
            f += 2 * oh * ow * c.cout * c.k * c.k * c.cin
        for d in self.dense_layers():
            f += 2 * d.fin * d.fout
        return f


def _out(n: int, k: int, s: int, padding: str) -> int:
    if padding == 'SAME':
        return -(-n // s)
    return (n - k) // s + 1


def _tf_pads(n: int, out: int, k: int, s: int, padding: str) -> Tuple[int, int]:
    if padding == 'VALID':
        return (0, 0)
    total = max((out - 1) * s + k - n, 0)
    return (total // 2, total - total // 2)


def _conv_stack(input_shape, layers, padding, pool) -> Tuple[ConvSpec, ...]:
    h, w, c = input_shape
    convs = []
    for name, k, s, cout in layers:
        spec = ConvSpec(name, k, s, c, cout, padding, pool, (h, w))
        convs.append(spec)
        (h, w), c = spec.out_hw, cout
    return tuple(convs)


def build_arch(network: str, input_shape: Sequence[int], num_actions: int, *,
               dueling: bool = False, distributional: bool = False, num_atoms: int = 51,
               v_min: float = -10.0, v_max: float = 10.0, noisy: bool = False,
               noisy_sigma0: float = 0.5) -> ArchSpec:
    input_shape = tuple(int(x) for x in input_shape)
    atoms = num_atoms if distributional else 1
    A = num_actions
    if network == 'simple':
        if len(input_shape) != 1:
            raise RuntimeError('SimpleNetwork expects 1-d input')
        trunk = (DenseSpec('hidden1', input_shape[0], 20, 'tanh'),
                 DenseSpec('hidden2', 20, 20, 'tanh'))
        if dueling:
            value = (DenseSpec('value/output', 20, atoms, None, noisy=noisy),)
            head = (DenseSpec('advantage/output', 20, A * atoms, None, noisy=noisy),)
        else:
            value = ()
            head = (DenseSpec('output', 20, A * atoms, None, noisy=noisy),)
        return ArchSpec(network, input_shape, A, (), trunk, head, value, atoms, v_min, v_max, noisy, noisy_sigma0)

    if len(input_shape) != 3:
        raise RuntimeError('%s expects 3-d input (H, W, frames)' % network)
    if network == 'cnn':
        convs = _conv_stack(input_shape, [('conv1', 8, 4, 32), ('conv2', 4, 2, 64), ('conv3', 3, 1, 64)],
                            'SAME', True)
        hidden = 256
        flat = convs[-1].out_hw[0] * convs[-1].out_hw[1] * convs[-1].cout
        if flat != 256:
            # The reference hard-codes reshape([-1, 256]) (network.py:333,401) and
            # silently mis-batches other input sizes; we refuse instead.
            raise RuntimeError('cnn requires inputs that pool down to 2x2x64 (e.g. 84x84); got flatten=%d' % flat)
    elif network == 'nature':
        convs = _conv_stack(input_shape, [('conv1', 8, 4, 32), ('conv2', 4, 2, 64), ('conv3', 3, 1, 64)],
                            'VALID', False)
        hidden = 512
    else:
        raise RuntimeError('Unsupported network type {}'.format(network))
    flat = convs[-1].out_hw[0] * convs[-1].out_hw[1] * convs[-1].cout
    if dueling:
        value = (DenseSpec('value/fcl', flat, hidden, 'relu', noisy=noisy),
                 DenseSpec('value/output', hidden, atoms, None, noisy=noisy))
        head = (DenseSpec('advantage/fcl', flat, hidden, 'relu', noisy=noisy),
                DenseSpec('advantage/output', hidden, A * atoms, None, noisy=noisy))
    else:
        value = ()
        head = (DenseSpec('fcl', flat, hidden, 'relu', noisy=noisy),
                DenseSpec('output', hidden, A * atoms, None, noisy=noisy))
    return ArchSpec(network, input_shape, A, convs, (), head, value, atoms, v_min, v_max, noisy, noisy_sigma0)


def arch_from_config(config, input_shape, num_actions) -> ArchSpec:
    return build_arch(config.network, input_shape, num_actions,
                      dueling=config.dueling, distributional=config.distributional,
                      num_atoms=config.num_atoms, v_min=config.v_min, v_max=config.v_max,
                      noisy=config.noisy, noisy_sigma0=config.noisy_sigma0)

"""Tuning constants of the HIP executor's launches (``--kernel_tuning``).

One documented place for the knobs that earlier rounds read from the environment inside the
launch path (DQN_WG_CHUNKS, DQN_DEP_AT, DQN_FOLD_TWO_PER_CU, DQN_TFACT). They are now fixed when
the executor is built, from the run configuration:

    --kernel_tuning "wg_conv_chunks=3,dep_at=-1,fold_two_per_cu=1,tfact=0"

Every default is the measured best on MI355X; the measurements are cited per field. Knobs that
lost their A/B (fc jobs interleaved with the weight-gradient tiles, acquire-fenced dependent jobs,
sc1 slot loads in the head fold) were removed from the kernels instead.
"""
from __future__ import annotations

import dataclasses


@dataclasses.dataclass(frozen=True)
class KernelTuning:
    # row chunks (128 rows; 64 in the fp32 build) per conv weight-gradient tile of the fused wgrad +
    # update launch (summed in registers, one set of fp32 atomics per tile). -1 = the measured best
    # per net and build: Nature bf16 3 x 128 rows -- 3 > 2 > 4 on the flagship (15.33k / 15.04k /
    # 14.76k SGD steps/s, profiles/r5_late_ab.md; again after the round-6 tile loads: 15.40-15.55k /
    # 15.06-15.09k / 14.97k) --, Nature fp32 4 x 64 (10.13-10.19k vs 9.91k at 6, 10.14k at 5, 9.92-9.96k
    # at 3, 9.47k at 2, profiles/r6_ab_wg_chunks_late.jsonl); the reference `cnn` 256 rows -- bf16 2 > 3
    # (18.52k / 17.43k; round 6 earlier: 2 > 1 > 3 > 6, profiles/r6_ab_wg_chunks.jsonl), fp32 4 > 3 > 6 > 2
    # (11.66-11.67k / 11.45k / 10.75k / 10.80k)
    wg_conv_chunks: int = -1
    # grid position of the range-dependent update jobs of that launch: after the first ``dep_at`` fc
    # jobs; -1 = the measured policy (noisy nets: after 500 of their ~1.6k fc jobs, +0.3-1.0 % over
    # 300 in 4 of 4 rounds; plain nets: at the end, 0 / 150 / 400 measured no better)
    dep_at: int = -1
    # head fold (fc_head.hip) in spin mode may run two blocks per CU when one per CU cannot hold
    # the grid (dueling / 3-instance launches; round 5, commit 69b1367)
    fold_two_per_cu: int = 1
    # noisy C51 nets: the target keeps separate mu / sigma fc fragments written only at a sync and
    # mixes its noise inside the fc forward. Measured slower (optimizer 58.4 -> 53.2 us but the fc
    # forward 10.5 -> 20.0 us: 7.29k -> 7.04k SGD steps/s, profiles/r5_late_ab.md), so opt-in
    tfact: int = 0
    # reference `cnn` backward: workgroups per sample (1, 2 or 4: the conv2 dgrad m-tiles and pool1
    # windows split over them; 4 also halves each wave's K range). -1 = 4, the measured best in both
    # builds: fp32 9.13k / 9.98k / 10.56k, bf16 17.41k / 17.99k / 18.61k SGD steps/s for 1 / 2 / 4
    # (`--variant ref`, profiles/r6_ab_cnn_bwd_parts.jsonl)
    cnn_bwd_parts: int = -1

    @classmethod
    def parse(cls, spec: str = '') -> 'KernelTuning':
        """``"key=value,key=value"`` (empty: the defaults); unknown keys raise."""
        kw = {}
        names = {f.name for f in dataclasses.fields(cls)}
        for part in (spec or '').replace(' ', '').split(','):
            if not part:
                continue
            k, _, v = part.partition('=')
            if k not in names:
                raise ValueError('--kernel_tuning: unknown key %r (known: %s)' % (k, sorted(names)))
            kw[k] = int(v)
        t = cls(**kw)
        if t.wg_conv_chunks != -1 and not 1 <= t.wg_conv_chunks <= 8:
            raise ValueError('--kernel_tuning: wg_conv_chunks -1 (auto) or in [1, 8]')
        if t.cnn_bwd_parts not in (-1, 1, 2, 4):
            raise ValueError('--kernel_tuning: cnn_bwd_parts -1 (auto), 1, 2 or 4')
        return t

    def cnn_parts(self, dtype: str) -> int:
        """Workgroups per sample of the reference cnn's fused backward (``cnn_bwd_parts``, -1 resolved)."""
        if self.cnn_bwd_parts > 0:
            return self.cnn_bwd_parts
        return 4

    def conv_chunks(self, network: str, dtype: str) -> int:
        """Row chunks per fused conv weight-gradient tile (``wg_conv_chunks``, -1 resolved)."""
        if self.wg_conv_chunks > 0:
            return self.wg_conv_chunks
        if dtype == 'fp32':
            return 4                                   # (4 x 64 rows, both nets)
        return 2 if network == 'cnn' else 3

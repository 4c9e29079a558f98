"""Probe: the fused weight-gradient + optimizer launch (executor._update_split) of the flagship
step, timed alone (HIP events over back-to-back launches):

  wgrad_group      the grouped weight-gradient launch it replaces (256-row chunks)
  F                the fused launch: lead block, weight-gradient tiles, fc jobs, dependent jobs
  F_nosampler      the same without the next-minibatch block
  F_fc_only        the fc jobs alone (FcFuse launch, no weight-gradient tiles)
  fused_old        the previous update launch (every job, sampler block; gradients read)

    python scripts/probe_split.py [--iters 200] [extra config flags...]

Prints one JSON line of mean us per launch.
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from dist_dqn_amd.config import preset
    from dist_dqn_amd.learner import Learner
    from dist_dqn_amd.models.network import Network
    from dist_dqn_amd.optim import kernel_op
    from dist_dqn_amd.replay import DeviceReplay
    args = sys.argv[1:]
    iters = 200
    if args[:1] == ['--iters']:
        iters, args = int(args[1]), args[2:]
    real_only = args[:1] == ['--real-only']     # only the learner's own launch (e.g. Rainbow's noisy / PER args)
    if real_only:
        args = args[1:]
    dev = torch.device('cuda', 0)
    cfg = preset('nature', 'Pong-v0', '--seed=0 --dtype=bf16 --replay_memory_capacity=65536 ' + ' '.join(args))
    net = Network.create_network(cfg, (84, 84, 4), 6, device=dev)
    rep = DeviceReplay(65536, (84, 84), 4, device=dev, prioritized=cfg.prioritized_replay)
    rep.fill_synthetic(65536, 6)
    learner = Learner(net, rep, cfg, use_graph=False)
    assert learner._defer_wgrad, 'the split update is not active for this config'
    ex = net.executor
    seen = {}
    orig = ex._update_split

    def spy(*a, **k):
        seen['wg'], seen['fc'] = ex._wg_pending, ex._fc_pending
        return orig(*a, **k)

    ex._update_split = spy
    for _ in range(3):
        learner.step()
    torch.cuda.synchronize()
    ex._update_split = orig
    wg, fc = seen['wg'], seen['fc']
    members, dims, scales = wg
    opt = net.optimizer
    hp = opt.hp
    hps = [float(hp[k]) for k in ('momentum', 'rho', 'rms_mom', 'rms_eps', 'b1', 'b2', 'adam_eps', 'ad_rho', 'ad_eps')]
    plan, nwg, jobs, nfc = ex._wg_plan(wg, net.grad, dev)[:4]
    nint = ex.ext.UPD_JOB_INTS
    jf = jobs[:nfc * nint]
    s0 = opt.slots[0] if opt.slots else net.online.flat
    s1 = opt.slots[1] if len(opt.slots) > 1 else net.online.flat
    base = (net.online.flat, net.grad, s0, s1, opt.beta_powers, opt.ticket, float(opt.lr), float(opt.reg_param),
            int(opt.layout.reg_end), 1.0, net.global_step, hps)
    p, pt = ex.packed(net.online.flat), ex.packed(net.target.flat)
    fca = [int(fc[0]), int(fc[1]), int(fc[2]), ex.FLAT, ex.HH]
    smp = []                              # (prioritized: the sampler block runs the PER step instead)
    if not cfg.prioritized_replay:
        spec = rep.next_sample_spec(32)
        smp = list(spec['spec']) + [int(spec['B'])] if spec['kind'] == 'uniform' else []
    op = kernel_op(opt)

    def launch(jobs, fcx, wgp=0, nb=0, sample=()):
        ex.ext.optim_pack(op, *base, jobs, p, net.target.flat, pt, 1 << 30, ex.opt_max_grid, None, None, None, None,
                          list(sample), [], [], None, None, None, None, fcx, 0, wg=wgp, wg_blocks=nb)

    def timeit(fn):
        for _ in range(10):
            fn()
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(iters):
            fn()
        b.record()
        torch.cuda.synchronize()
        return round(a.elapsed_time(b) * 1000.0 / iters, 2)

    out = {'wg_blocks': nwg, 'fc_jobs': nfc, 'jobs': jobs.numel() // nint}
    if os.environ.get('DQN_OPT_PROF'):
        # the learner's own update launch (its real noise / PER / target-mix arguments), eager step
        for _ in range(3):
            out['timeline_real_us'] = timeline(ex, plan, nwg, jobs, nfc, nint, learner.step)
    if real_only:
        print(json.dumps(out))
        return
    out['wgrad_group'] = timeit(lambda: ex.ext.qnet_wgrad_group(members, dims, scales))
    out['F'] = timeit(lambda: launch(jobs, fca, plan.data_ptr(), nwg, sample=smp))
    out['F_nosampler'] = timeit(lambda: launch(jobs, fca, plan.data_ptr(), nwg))
    out['F_fc_only'] = timeit(lambda: launch(jf, fca))
    # (the previous single launch reads every gradient from the flat buffer: fc jobs as well)
    jall = ex._upd_jobs(dev)
    out['fused_old'] = timeit(lambda: launch(jall, fca, sample=smp))
    for cc in (2, 4):                     # chunks per conv tile (the executor default: 3)
        ex.wg_conv_chunks = cc
        ex._wg_plans = {}
        pl2, n2, j2 = ex._wg_plan(wg, net.grad, dev)[:3]
        out['F_chunks%d' % cc] = timeit(lambda: launch(j2, fca, pl2.data_ptr(), n2, sample=smp))
        out['wg_blocks_chunks%d' % cc] = n2
    ex.wg_conv_chunks = 3
    ex._wg_plans = {}
    plan, nwg, jobs, nfc = ex._wg_plan(wg, net.grad, dev)[:4]
    if os.environ.get('DQN_OPT_PROF'):
        out['timeline_us'] = timeline(ex, plan, nwg, jobs, nfc, nint, lambda: launch(jobs, fca, plan.data_ptr(), nwg,
                                                                                 sample=smp))
        # the fc jobs alone (no tiles, no lead block's sampler): their start spread = how fast the
        # launch gets its blocks onto the CUs
        t = timeline_fc_only(ex, nfc, lambda: launch(jf, fca))
        out['timeline_fc_only_us'] = t
        # phases inside the tiles of that launch (us after each tile's start): staged chunk 0 |
        # chunk 0 MFMAs | staged chunk 1 | chunk 1 MFMAs | results issued | drained
        ph = ex.ext.optim_tile_phases(min(nwg, 512))
        rows = [[(ph[8 * b + i] - ph[8 * b]) / 100.0 if ph[8 * b + i] else None for i in (1, 2, 3, 4, 6, 7)]
                for b in range(len(ph) // 8)]
        mem = [int(m[0]) for m in members]
        def med(v):
            v = sorted(x for x in v if x is not None)
            return round(v[len(v) // 2], 2) if v else None
        bounds, lo = [], 0
        for m in members:
            pass
        # per member (the timeline's ready word holds a tile's member id)
        tlv = ex.ext.optim_timeline(1 + len(rows))
        per = {}
        for b, r in enumerate(rows):
            per.setdefault(int(tlv[3 * (b + 1) + 1]), []).append(r)
        out['tile_phases_us'] = {'first_conv1_tiles': rows[:3],
                                 'median_all': [med([r[i] for r in rows]) for i in range(6)],
                                 'median_by_member': {str(m): {'n': len(v), 'phases': [med([r[i] for r in v])
                                                                                         for i in range(6)]}
                                                      for m, v in sorted(per.items())}}
    print(json.dumps(out))


def timeline_fc_only(ex, nfc, fn):
    """Start / duration / end percentiles of the blocks of a launch of fc jobs only."""
    import torch
    fn()
    torch.cuda.synchronize()
    t = ex.ext.optim_timeline(nfc + 1)
    st = [t[3 * b] for b in range(nfc + 1) if t[3 * b]]
    t0 = min(st)
    pct = lambda v: [round(sorted(v)[int(q * (len(v) - 1))], 2) for q in (0.0, 0.25, 0.5, 0.75, 1.0)]
    rows = [(t[3 * b], t[3 * b + 2]) for b in range(nfc + 1) if t[3 * b]]
    out = {'start': pct([(a - t0) / 100.0 for a, _ in rows]), 'dur': pct([(e - a) / 100.0 for a, e in rows]),
           'end': pct([(e - t0) / 100.0 for _, e in rows]), 'blocks': len(rows)}
    return out


def timeline(ex, plan, nwg, jobs, nfc, nint, fn):
    """Per-block [start, ready, end] (us from the first start) of one launch, summarised: the lead
    block, each weight-gradient member (start / duration / end percentiles), the fc jobs, the
    dependent jobs."""
    import torch
    if True:
        fn()
        torch.cuda.synchronize()
        ngrid = 1 + nwg + jobs.numel() // nint
        t = ex.ext.optim_timeline(ngrid)
        st = [t[3 * b] for b in range(ngrid)]
        t0 = min(st)
        us = lambda v: round((v - t0) / 100.0, 2)          # s_memrealtime: 100 MHz
        tl = {'lead': [us(t[0]), us(t[1]) if t[1] else None, us(t[2])]}
        pct = lambda v: [round(sorted(v)[int(q * (len(v) - 1))], 2) for q in (0.0, 0.5, 1.0)]
        mem = {}
        for b in range(1, 1 + nwg):
            mem.setdefault(int(t[3 * b + 1]), []).append((us(t[3 * b]), (t[3 * b + 2] - t[3 * b]) / 100.0,
                                                          us(t[3 * b + 2])))
        tl['members'] = {str(m): {'n': len(v), 'start': pct([x[0] for x in v]), 'dur': pct([x[1] for x in v]),
                                  'end': pct([x[2] for x in v])} for m, v in sorted(mem.items())}
        fcb = range(1 + nwg, 1 + nwg + nfc)
        tl['fc_jobs'] = {'start': pct([us(t[3 * b]) for b in fcb]), 'dur': pct([(t[3 * b + 2] - t[3 * b]) / 100.0
                                                                                for b in fcb]),
                         'end': pct([us(t[3 * b + 2]) for b in fcb])}
        dep = range(1 + nwg + nfc, ngrid)
        if len(dep):
            tl['dep_jobs'] = {'start': pct([us(t[3 * b]) for b in dep]), 'ready': pct([us(t[3 * b + 1]) for b in dep]),
                              'end': pct([us(t[3 * b + 2]) for b in dep])}
        return tl


if __name__ == '__main__':
    main()

"""Probe: the fused optimizer+pack launch (csrc/kernels/optim.hip optim_pack_kernel) timed alone,
per variant, on the flagship Nature-CNN (1.69M parameters, RMSProp at momentum 0):

  plain      gradient read from the flat fp32 buffer (mode 0)
  fc_fused   fc weight / bias gradient formed in-launch from the fc rows (FcFuse, mode 8)
  +sampler   one extra block drawing the next uniform minibatch
  +mom       the deferred RMSProp mom slot stored (request_slots)
  sgd        SGD: weights only (the byte floor of an update)

    python scripts/probe_optim.py [--iters 200]

Prints one JSON line of mean us per launch (CUDA events around back-to-back launches).
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--iters', type=int, default=200)
    args = ap.parse_args()
    import torch
    from dist_dqn_amd.config import preset
    from dist_dqn_amd.learner import Learner
    from dist_dqn_amd.models.network import Network
    from dist_dqn_amd.replay import DeviceReplay
    dev = torch.device('cuda', 0)
    out = {}
    for opt_name in ('rmsprop', 'sgd'):
        cfg = preset('nature', 'Pong-v0', '--seed=0 --dtype=bf16 --replay_memory_capacity=65536 --optimizer=%s'
                     % opt_name)
        net = Network.create_network(cfg, (84, 84, 4), 6, device=dev)
        rep = DeviceReplay(65536, (84, 84), 4, device=dev)
        rep.fill_synthetic(65536, 6)
        learner = Learner(net, rep, cfg, use_graph=False)
        for _ in range(3):
            learner.step()
        ex = net.executor
        ws = ex._workspace(32, dev)
        fc = (ws['x3'][0].data_ptr(), ws['dh'].data_ptr(), 32)
        spec = rep.next_sample_spec(32)

        def launch(fused, sampler):
            ex.update_and_pack(net.optimizer, net.online.flat, net.grad, 1.0, net.global_step,
                               target=net.target.flat, target_freq=1 << 30,
                               next_sample=spec if sampler else None, fc=fc if fused else None)
            if not fused:
                ex._fc_pending = None

        def timeit(fn):
            for _ in range(10):
                fn()
            torch.cuda.synchronize()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(args.iters):
                fn()
            b.record()
            torch.cuda.synchronize()
            return round(a.elapsed_time(b) * 1000.0 / args.iters, 2)

        if opt_name == 'sgd':
            out['sgd'] = timeit(lambda: launch(False, False))
            continue
        out['plain'] = timeit(lambda: launch(False, False))
        out['fc_fused'] = timeit(lambda: launch(True, False))
        out['plain+sampler'] = timeit(lambda: launch(False, True))
        out['fc_fused+sampler'] = timeit(lambda: launch(True, True))
        # the launch without the fc weight tiles (what remains if they run elsewhere)
        items_all = ex.upd_items
        ex.upd_items = [it for it in items_all if not (it[0] == 0 and it[20] >= 0)]
        ex._upd_dev = {}
        out['no_fc_tiles+sampler'] = timeit(lambda: launch(True, True))
        out['jobs_no_fc_tiles'] = len(ex.upd_items)
        ex.upd_items = items_all
        ex._upd_dev = {}
        if os.environ.get('DQN_OPT_PROF'):
            launch(True, True)
            torch.cuda.synchronize()
            t = ex.ext.optim_prof()
            out['stamps_block0'] = [t[i] - t[0] for i in range(1, 5)]
            out['stamps_block1'] = [t[8 + i] - t[8] if t[8 + i] else 0 for i in range(1, 8)]
        net.optimizer.request_slots(True)
        out['fc_fused+sampler+mom'] = timeit(lambda: launch(True, True))
        net.optimizer.request_slots(False)
        out['jobs'] = len(ex.upd_items)
    print(json.dumps(out), flush=True)


if __name__ == '__main__':
    main()

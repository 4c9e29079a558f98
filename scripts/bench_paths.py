"""User-path throughput: the two ways ``python -m dist_dqn_amd`` trains an Atari id on one GPU,
measured through the real CLI entry (`cli.run_worker`), not the benchmark harness.

    python scripts/bench_paths.py --path host   --steps 2000   # dqn_single_node.sh atari Pong-v0
    python scripts/bench_paths.py --path device --steps 20000  # ... --device_envs=4

* ``host``: the reference agent loop (`/root/reference/src/dqn_agent.py:72-106`): one env on the
  host (SyntheticAtariEnv frames through the C++ preprocessing), a batch-1 greedy forward per
  acting step, an SGD step every ``update_freq`` env steps (HIP learner, HBM replay);
* ``device``: ``--device_envs=4`` GPU-resident envs acting inside the learner's launches (what
  bench.py times), under the same supervisor / checkpoint / metrics code.

Prints one JSON line: SGD steps/s and env frames/s over the run after prefill.
"""
import argparse
import json
import os
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--path', choices=['host', 'device'], default='device')
    ap.add_argument('--steps', type=int, default=2000, help='SGD steps (--max_train_steps)')
    ap.add_argument('--extra', default='')
    args = ap.parse_args()
    from dist_dqn_amd.cli import run_worker
    from dist_dqn_amd.config import preset
    logdir = tempfile.mkdtemp(prefix='bench_paths_')
    flags = ('--device=cuda --replay_memory_capacity=200000 --replay_start_size=10000 --checkpoint_secs=0 '
             '--max_train_steps=%d --logdir=%s --log_level=WARNING %s' % (args.steps, logdir, args.extra))
    if args.path == 'device':
        flags += ' --device_envs=4'
    cfg = preset('atari', 'Pong-v0', flags)
    t0 = time.perf_counter()
    out = run_worker(cfg)
    el = time.perf_counter() - t0
    recs = [json.loads(line) for line in open(os.path.join(logdir, 'metrics.rank0.jsonl'))]
    res = {'path': args.path, 'sgd_steps': args.steps, 'wall_s': round(el, 2),
           'network': cfg.network, 'executor': None, 'env': cfg.env}
    if args.path == 'device':
        done = [r for r in recs if r.get('kind') == 'done'][-1]
        res.update(sgd_steps_per_sec=round(done['sgd_steps_per_sec'], 1),
                   env_frames_per_sec=round(done['env_frames_per_sec'], 1), executor=out.net.executor.name)
    else:
        eps = [r for r in recs if r.get('kind') == 'episode']
        agent = out
        # rates over the whole run after prefill (the agent's meters start after the prefill)
        frames = agent.frame_meter.count
        span = time.perf_counter() - agent.t_train0
        res.update(sgd_steps_per_sec=round(agent.training_steps / span, 1), env_frames_per_sec=round(frames / span, 1),
                   episodes=len(eps), executor=agent.network.executor.name)
    print(json.dumps(res), flush=True)


if __name__ == '__main__':
    main()

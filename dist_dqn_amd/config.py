"""Flag table, presets and the run configuration object.

Flag names, defaults and choices are kept identical to the reference CLI
(`/root/reference/src/main.py:12-98`) so a reference command line parses
unchanged; presets mirror `/root/reference/scripts/dqn_params.sh:7-42`.
Flags after the ``# --- extensions`` marker are new (north-star features:
Huber/Double/Dueling/PER/soft target/C51/noisy, bf16, RCCL DP, Ape-X actors).
"""
from __future__ import annotations

import argparse
import dataclasses
import shlex
from typing import List, Optional, Sequence

OPTIMIZERS = ['adadelta', 'adagrad', 'adam', 'ftrl', 'sgd', 'momentum', 'rmsprop']
NETWORKS = ['simple', 'cnn', 'nature']

# Reference presets (scripts/dqn_params.sh:7-20 and :24-42).
CONTROL = (
    "--network=simple --optimizer=adam --lr=0.001 --minibatch_size=100 "
    "--num_episodes=10000 --max_steps_per_episode=200 "
    "--replay_memory_capacity=50000 --target_update_freq=3000 "
    "--reward_discount=0.9 --init_random_action_prob=0.5 "
    "--min_random_action_prob=0.1 --random_action_explore_steps=50000"
)
ATARI = (
    "--network=cnn --optimizer=rmsprop --lr=0.00025 --minibatch_size=32 "
    "--num_episodes=10000 --max_steps_per_episode=500000 "
    "--replay_memory_capacity=1000000 --target_update_freq=10000 "
    "--reward_discount=0.99 --init_random_action_prob=1.0 "
    "--min_random_action_prob=0.1 --random_action_explore_steps=1000000 "
    "--frames_per_state=4 --update_freq=4 --replay_start_size=10000 "
    "--resize_width=84 --resize_height=84"
)
# North-star presets (BASELINE.json "configs": Nature-CNN in bf16, Rainbow on the fp16 MFMA
# path). The reference presets above keep the reference's fp32 (--dtype default).
NATURE = ATARI.replace("--network=cnn", "--network=nature") + " --input_scale=0.00392156862745098 --dtype=bf16"
DOUBLE_DUELING = NATURE + " --double_dqn --dueling --loss=huber"
APEX = DOUBLE_DUELING + " --prioritized_replay --n_step=3 --num_actors=256"
RAINBOW = (NATURE + " --double_dqn --dueling --distributional --noisy --prioritized_replay --n_step=3 --optimizer=adam "
           "--lr=0.0000625").replace("--dtype=bf16", "--dtype=fp16")

PRESETS = {
    'control': CONTROL,
    'atari': ATARI,
    'nature': NATURE,
    'double_dueling': DOUBLE_DUELING,
    'apex': APEX,
    'rainbow': RAINBOW,
}


def dqn_params_for_env(env_type: str, env_name: str) -> str:
    """Equivalent of `dqn_params_for_env` (scripts/dqn_params.sh:44-64)."""
    if env_type not in PRESETS:
        raise ValueError('Invalid env_type %s. Choices are %s.' % (env_type, sorted(PRESETS)))
    return '--env=%s %s' % (env_name, PRESETS[env_type])


def build_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(prog='dist_dqn_amd')
    a = p.add_argument
    a('--log_level', default='INFO', help='Log verbosity')
    # Environment
    a('--env', default='CartPole-v0', help='Environment name')
    a('--monitor', action='store_true', help='Write per-episode monitor stats')
    a('--monitor_path', default='/tmp/gym', help='Path for monitor logs')
    a('--disable_video', action='store_true', help='Accepted for parity (no video)')
    # Network
    a('--network', default='simple', choices=NETWORKS, help='Network architecture type')
    a('--lr', default=0.001, type=float, help='Learning rate')
    a('--reg_param', default=0.001, type=float, help='Regularization param')
    a('--optimizer', default='sgd', choices=OPTIMIZERS, help='Optimizer')
    a('--momentum', default=0.9, type=float, help='Momentum for MomentumOptimizer')
    a('--rmsprop_decay', default=0.95, type=float, help='Decay for RMSProp')
    # Agent
    a('--num_episodes', default=10000, type=int)
    a('--max_steps_per_episode', default=1000, type=int)
    a('--minibatch_size', default=30, type=int)
    a('--frames_per_state', default=1, type=int)
    a('--resize_width', default=0, type=int)
    a('--resize_height', default=0, type=int)
    a('--reward_discount', default=0.9, type=float)
    a('--replay_memory_capacity', default=10000, type=int)
    a('--replay_start_size', default=0, type=int)
    a('--init_random_action_prob', default=0.9, type=float)
    a('--min_random_action_prob', default=0.1, type=float)
    a('--random_action_explore_steps', default=10000, type=int)
    a('--update_freq', default=1, type=int)
    a('--target_update_freq', default=10000, type=int)
    # Distribution
    a('--ps_hosts', default='', help='Accepted for parity; mapped onto ranks')
    a('--worker_hosts', default='localhost:0', help='Comma separated host:port list')
    a('--job', default='worker', choices=['ps', 'worker'])
    a('--task_id', default=0, type=int)
    a('--gpu_id', default=0, type=int)
    a('--sync', action='store_true', help='Synchronous data parallel training')
    a('--disable_cpu_param_pinning', action='store_true')
    a('--disable_target_replication', action='store_true')
    # Summary
    a('--logdir', default='/tmp/train_logs')
    a('--summary_freq', default=100, type=int)

    # --- extensions (not in the reference) ---------------------------------
    a('--seed', default=None, type=int, help='Global RNG seed')
    a('--device', default='auto', choices=['auto', 'cpu', 'cuda'])
    a('--backend', default='auto', choices=['auto', 'hip', 'torch'],
      help='Learner executor: hand-written HIP kernels or the torch oracle')
    a('--dtype', default='fp32', choices=['fp32', 'bf16', 'fp16'],
      help='Compute dtype of the MFMA network kernels (fp32 master weights always; the HIP executor '
           'computes in bf16 unless fp16 is asked for)')
    a('--input_scale', default=1.0, type=float,
      help='Multiplier on raw uint8 pixels (reference: 1.0, i.e. no /255)')
    a('--loss', default='mse', choices=['mse', 'huber'])
    a('--huber_delta', default=1.0, type=float)
    a('--double_dqn', action='store_true')
    a('--dueling', action='store_true')
    a('--distributional', action='store_true', help='C51 head')
    a('--num_atoms', default=51, type=int)
    a('--v_min', default=-10.0, type=float)
    a('--v_max', default=10.0, type=float)
    a('--noisy', action='store_true', help='Factorised-Gaussian noisy FC layers')
    a('--noisy_sigma0', default=0.5, type=float)
    a('--target_update_tau', default=1.0, type=float,
      help='1.0 = hard copy every target_update_freq; <1 = Polyak every step')
    a('--n_step', default=1, type=int)
    a('--reward_clip', default=0.0, type=float, help='0 disables clipping')
    a('--prioritized_replay', action='store_true')
    a('--per_alpha', default=0.6, type=float)
    a('--per_beta0', default=0.4, type=float)
    a('--per_beta_steps', default=1000000, type=int)
    a('--per_eps', default=1e-6, type=float)
    a('--num_actors', default=1, type=int, help='Ape-X actor count')
    a('--actor_param_sync_freq', default=400, type=int,
      help='Ape-X: learner steps between the inference service\'s parameter snapshots (0 = live weights)')
    a('--apex_eps_base', default=0.4, type=float, help='Ape-X per-actor epsilon base')
    a('--apex_eps_alpha', default=7.0, type=float, help='Ape-X per-actor epsilon exponent spread')
    a('--apex_ring', default=1024, type=int, help='Ape-X transition ring capacity per actor (records)')
    a('--apex_seconds', default=0.0, type=float,
      help='Ape-X: wall-clock budget of the run (0 = none); under sync DP a coordinated stop')
    a('--apex_native_serve', default=1, type=int,
      help='Ape-X: answer the actors from a C++ thread replaying captured inference graphs (GPU)')
    a('--device_envs', default=0, type=int,
      help='Synthetic Atari ids on a GPU: run this many GPU-resident envs whose acting step rides inside '
           'the learner\'s launches (fused acting; the path bench.py measures) instead of the host agent '
           'loop. update_freq / device_envs acting steps per SGD step; runs until --max_train_steps or a '
           'stop request')
    a('--device_graph_steps', default=8, type=int,
      help='--device_envs (one process): SGD steps per replayed HIP graph')
    a('--apex_native_ingest', default=1, type=int,
      help='Ape-X (GPU, image envs): move the actors\' ring records into the HBM replay from a C++ thread '
           '(csrc/ingest_server.cpp) instead of the learner\'s Python thread')
    a('--apex_reserve_cpus', default=3, type=int,
      help='Ape-X: CPUs reserved for the learner, ingest and inference threads (one each; the actor '
           'processes run on the rest); 0 = no pinning')
    a('--apex_pace', default=0.9, type=float,
      help='Ape-X under a CFS CPU quota smaller than the visible CPUs: > 0 = unpinned actors paced so '
           'their CPU time together stays under this fraction of (quota - reserved CPUs) (measured, 256 '
           'actors on a 16-CPU quota: learner 8.4k SGD steps/s at 0.9 vs 0.8k with pinning); '
           '0 = pin the actors to quota-many CPU ids and reserve CPUs for the learner threads')
    a('--apex_graph_steps', default=4, type=int,
      help='Ape-X learner: SGD steps per replayed HIP graph (one host call per that many steps)')
    a('--apex_serve_gap_us', default=100, type=int,
      help='Ape-X inference service: pause after each served batch (us) so requests batch up and the '
           'learner loop gets the GIL')
    a('--allreduce', default='auto', choices=['auto', 'rccl', 'xgmi'],
      help='gradient all-reduce transport: RCCL, the peer-to-peer xGMI kernel (in-graph), or auto '
           '(self-test + time both at start-up, keep the faster)')
    a('--allreduce_dtype', default='fp32', choices=['fp32', 'bf16'],
      help='wire dtype of the gradient all-reduce (bf16 halves the bytes; optimizer stays fp32)')
    a('--grad_bucket_mb', default=64.0, type=float,
      help='all-reduce bucket size; the default keeps the whole flat gradient in ONE collective')
    a('--overlap_allreduce', default=1, type=int,
      help='DP: all-reduce the dense-layer gradients while the conv backward runs (two collectives)')
    a('--lowrank_dense', default=1, type=int,
      help='DP over xgmi: exchange the fc layer\'s gradient factors (its input rows and dL/dh rows, '
           'all-gathered) and form the summed fc weight gradient on every rank, instead of '
           'all-reducing the full fc gradient (exact; ~14x fewer bytes for Nature-CNN at B=32)')
    a('--hip_graph', default=1, type=int, help='Capture the learner step in a HIP graph')
    a('--fuse_sampling', default=2, type=int, choices=[0, 1, 2],
      help='Uniform GPU replay: 0 = sampler launch per step, 1 = the Nature trunk draws the minibatch, '
           '2 = the previous step\'s optimizer launch draws it (one extra block, off the critical path)')
    a('--summary_secs', default=120.0, type=float,
      help='chief: seconds between global_step/sec summaries (TF Supervisor step counter: 120)')
    a('--ps_timeout_s', default=60.0, type=float,
      help='async PS over xGMI: a worker pull that waits longer for the server flags an error (the '
           'learner raises at its next device check) instead of hanging')
    a('--fold_head', default=1, type=int,
      help='HIP executor, scalar heads: fc forward + output layer + TD loss + dQ / dH (+ the fused acting '
           'step) in ONE launch (csrc/kernels/fc_head.hip) instead of the fc launch + the head launch')
    a('--chain_dgrad', default=0, type=int,
      help='HIP executor, Nature net: 1 = the fc and conv3 data gradients in ONE launch whose stages wait on '
           'per-sample counters (dgrad_chain_kernel; 2: the conv2 dgrad too); 0 (default: measured faster) = '
           'separate launches')
    a('--fuse_fc_wgrad', default=1, type=int,
      help='HIP executor (16-bit builds): form the fc weight gradient (X^T dH, rank <= B) inside the '
           'fused optimizer launch instead of writing and re-reading it as an fp32 gradient')
    a('--fuse_wgrad_update', default=1, type=int,
      help='HIP executor (one process, 16-bit builds, with --fuse_fc_wgrad): compute the conv / '
           'output-layer weight gradients in the leading blocks of the fused optimizer\'s first '
           'launch, beside the fc update, instead of a launch of their own before it')
    a('--det_wgrad', default=0, type=int,
      help='HIP executor (one process, 16-bit builds): conv weight gradients as deterministic '
           'chunk-group partials summed in a fixed order by the fused optimizer launch (no fp32 '
           'atomics: bit-reproducible steps; measured 79.6 vs 71.4 us per flagship step, so opt-in)')
    a('--kernel_tuning', default='',
      help='HIP executor tuning constants, "key=value,..." (ops/tuning.py KernelTuning: wg_conv_chunks, '
           'dep_at, fold_two_per_cu, tfact); empty = the measured defaults')
    a('--checkpoint_secs', default=600, type=float,
      help='chief: seconds between periodic checkpoints (reference Supervisor: 600; <= 0 disables)')
    a('--max_to_keep', default=5, type=int)
    a('--save_agent_state', action='store_true', help='Checkpoint epsilon/step sidecar')
    a('--async_ps', action='store_true', help='Emulate async parameter-server updates')
    a('--ps_pipeline', default=0, type=int,
      help='async PS over xGMI: 1 = a worker takes the PS answer to its PREVIOUS push, then pushes this '
           'step\'s gradient and goes on (one more step of staleness, within the reference\'s Hogwild '
           'semantics; no per-step round trip to the server); 0 = push, then wait for this push\'s answer')
    a('--ps_lowrank', default=1, type=int,
      help='async PS over xGMI: push the fc weight gradient as its factors (fc input rows + dL/dh rows, rank '
           '<= B; the server forms it in its fused optimizer launch) instead of the 6.4 MB gradient')
    a('--ps_transport', default='auto', choices=['auto', 'p2p', 'xgmi'],
      help='--async_ps transport: one-sided xGMI peer memory (GPU; replicated targets) or '
           'torch.distributed point-to-point; auto = xgmi when available')
    a('--max_train_steps', default=0, type=int, help='Stop after N learner steps (0 = no limit)')
    a('--allreduce_check_steps', default=1000, type=int,
      help='xgmi transport: read its peer-timeout error word every N learner steps (host sync)')
    a('--stop_sync_steps', default=10, type=int,
      help='sync DP: ranks agree on a pending stop request every N train steps (CPU control plane)')
    a('--replica_check', default=1, type=int,
      help='sync DP: verify at the end of the run that every replica tensor is bit-identical')
    return p


@dataclasses.dataclass
class Config:
    """argparse-Namespace-compatible run configuration (attribute names = flag names)."""
    log_level: str = 'INFO'
    env: str = 'CartPole-v0'
    monitor: bool = False
    monitor_path: str = '/tmp/gym'
    disable_video: bool = False
    network: str = 'simple'
    lr: float = 0.001
    reg_param: float = 0.001
    optimizer: str = 'sgd'
    momentum: float = 0.9
    rmsprop_decay: float = 0.95
    num_episodes: int = 10000
    max_steps_per_episode: int = 1000
    minibatch_size: int = 30
    frames_per_state: int = 1
    resize_width: int = 0
    resize_height: int = 0
    reward_discount: float = 0.9
    replay_memory_capacity: int = 10000
    replay_start_size: int = 0
    init_random_action_prob: float = 0.9
    min_random_action_prob: float = 0.1
    random_action_explore_steps: int = 10000
    update_freq: int = 1
    target_update_freq: int = 10000
    ps_hosts: str = ''
    worker_hosts: str = 'localhost:0'
    job: str = 'worker'
    task_id: int = 0
    gpu_id: int = 0
    sync: bool = False
    disable_cpu_param_pinning: bool = False
    disable_target_replication: bool = False
    logdir: str = '/tmp/train_logs'
    summary_freq: int = 100
    seed: Optional[int] = None
    device: str = 'auto'
    backend: str = 'auto'
    dtype: str = 'fp32'
    input_scale: float = 1.0
    loss: str = 'mse'
    huber_delta: float = 1.0
    double_dqn: bool = False
    dueling: bool = False
    distributional: bool = False
    num_atoms: int = 51
    v_min: float = -10.0
    v_max: float = 10.0
    noisy: bool = False
    noisy_sigma0: float = 0.5
    target_update_tau: float = 1.0
    n_step: int = 1
    reward_clip: float = 0.0
    prioritized_replay: bool = False
    per_alpha: float = 0.6
    per_beta0: float = 0.4
    per_beta_steps: int = 1000000
    per_eps: float = 1e-6
    num_actors: int = 1
    actor_param_sync_freq: int = 400
    apex_eps_base: float = 0.4
    apex_eps_alpha: float = 7.0
    apex_ring: int = 1024
    apex_seconds: float = 0.0
    apex_serve_gap_us: int = 100
    apex_graph_steps: int = 4
    apex_native_ingest: int = 1
    apex_reserve_cpus: int = 3
    apex_pace: float = 0.9
    device_envs: int = 0
    device_graph_steps: int = 8
    apex_native_serve: int = 1
    allreduce: str = 'auto'
    allreduce_dtype: str = 'fp32'
    grad_bucket_mb: float = 64.0
    overlap_allreduce: int = 1
    lowrank_dense: int = 1
    hip_graph: int = 1
    fuse_sampling: int = 2
    fuse_fc_wgrad: int = 1
    fold_head: int = 1
    ps_timeout_s: float = 60.0
    chain_dgrad: int = 0
    fuse_wgrad_update: int = 1
    det_wgrad: int = 0
    kernel_tuning: str = ''
    summary_secs: float = 120.0
    checkpoint_secs: float = 600
    max_to_keep: int = 5
    save_agent_state: bool = False
    async_ps: bool = False
    ps_transport: str = 'auto'
    ps_pipeline: int = 0
    ps_lowrank: int = 1
    max_train_steps: int = 0
    allreduce_check_steps: int = 1000
    stop_sync_steps: int = 10
    replica_check: int = 1

    def replace(self, **kw) -> 'Config':
        return dataclasses.replace(self, **kw)

    @classmethod
    def from_namespace(cls, ns: argparse.Namespace) -> 'Config':
        names = {f.name for f in dataclasses.fields(cls)}
        return cls(**{k: v for k, v in vars(ns).items() if k in names})


def parse_args(argv: Optional[Sequence[str]] = None) -> Config:
    return Config.from_namespace(build_parser().parse_args(argv))


def preset(env_type: str, env_name: str, extra: str = '') -> Config:
    """Config for a preset, e.g. ``preset('atari', 'Pong-v0')``."""
    return parse_args(shlex.split(dqn_params_for_env(env_type, env_name) + ' ' + extra))


def defaults() -> Config:
    return parse_args([])


def flag_names() -> List[str]:
    return [a.dest for a in build_parser()._actions if a.dest != 'help']

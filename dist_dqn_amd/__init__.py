"""dist_dqn_amd — a distributed DQN training engine built for AMD MI355X (gfx950).

Capabilities of hbfs/dist-dqn (agent/train API, CLI flags and presets, MLP
and CNN Q-networks, replay, epsilon-greedy, target networks, multi-GPU
launch, TF-named checkpoints) re-designed MI355X-first: PyTorch-ROCm front
end, hand-written HIP/CDNA4 kernels for the learner's hot path, HBM-resident
replay, RCCL data parallelism over xGMI. See README.md / SURVEY.md.
"""
__version__ = '0.1.0'

from .config import Config, parse_args, preset  # noqa: F401,E402

"""reacherdistilation_amd -- MI355X-native batched Reacher-v2 rollout + policy distillation.

The hot path of winstonww/ReacherDistilation's src/distilation MLP training loop
(env.step/env.reset + teacher query + student MLP forward/backward + distillation loss +
Adam; reference mlp_train.py:143-204) as hand-written HIP kernels for gfx950 behind a
C ABI (include/reacher.h, include/reacher_distill.h), driven from Python on PyTorch-ROCm.
"""
from . import config  # noqa: F401

__all__ = ["config", "env", "policy", "distill"]

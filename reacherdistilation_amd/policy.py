"""Policy side of the hot path: parameter layout, initialisers and the teacher/student
objects the reference drivers hold.

Reference interfaces mirrored here:
  * ``TeacherAgent(env, sess, restore, batch)`` (reference teacher.py:12-20) wraps a
    baselines ppo1 ``MlpPolicy(hid_size=64, num_hid_layers=2)``: observation filter
    (RunningMeanStd, clip +-5) -> 2 x 64 tanh -> linear mean; state-independent logstd
    (``pi/pol/logstd`` in the reference's tfevents GraphDefs).  Its checkpoint
    (~/reacher/data/teacher.ckpt) is not in the reference repo, so the teacher here is
    synthetic: normc(1.0) hidden / normc(0.01) output from a seed, logstd fixed to the
    fixture's values (config.TEACHER_LOGSTD), filter mean 0 / std 1.
  * the student: the same MlpPolicy structure (BASELINE configs 2-5; reference
    backup/student_rollout.py:79-87 StudentAgent), logstd trainable, zero-initialised as
    in baselines' DiagGaussianPdType.
  * ``student_mlp_graph`` (reference student_nn.py:51-57): 16 -> 24 tanh -> 128 tanh ->
    128 -> 32 tanh -> 4 with glorot-uniform kernels; provided as a parameter container
    for the reference-shaped single-env driver (config 1), not run by the fused kernel.

Flat layout of an MlpPolicy (shared with include/reacher_distill.h and the kernels):
  W1[11][64] | b1[64] | W2[64][64] | b2[64] | W3[64][2] | b3[2] | logstd[2]   (P = 5060)
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np
import torch

from .config import ACSPACE_SHAPE, OBSPACE_SHAPE, PDFLAT_SHAPE, TEACHER_LOGSTD

OBD, HID, ACD = OBSPACE_SHAPE, 64, ACSPACE_SHAPE
P_W1 = 0
P_B1 = P_W1 + OBD * HID
P_W2 = P_B1 + HID
P_B2 = P_W2 + HID * HID
P_W3 = P_B2 + HID
P_B3 = P_W3 + HID * ACD
P_LS = P_B3 + ACD
P_TOT = P_LS + ACD          # 5060
SLICES = dict(W1=(P_W1, P_B1, (OBD, HID)), b1=(P_B1, P_W2, (HID,)), W2=(P_W2, P_B2, (HID, HID)),
              b2=(P_B2, P_W3, (HID,)), W3=(P_W3, P_B3, (HID, ACD)), b3=(P_B3, P_LS, (ACD,)),
              logstd=(P_LS, P_TOT, (ACD,)))


def normc(rng: np.random.RandomState, shape, std: float) -> np.ndarray:
    """baselines.common.tf_util.normc_initializer(std)."""
    out = rng.standard_normal(shape).astype(np.float32)
    out *= std / np.sqrt(np.square(out).sum(axis=0, keepdims=True))
    return out


@dataclass
class MlpPolicyParams:
    """A 2x64 MlpPolicy as one flat f32 vector plus its observation filter."""
    flat: np.ndarray                                   # [P_TOT] float32
    ob_mean: np.ndarray = field(default_factory=lambda: np.zeros(OBD, np.float32))
    ob_std: np.ndarray = field(default_factory=lambda: np.ones(OBD, np.float32))

    def __getitem__(self, name):
        a, b, shape = SLICES[name]
        return self.flat[a:b].reshape(shape)

    @classmethod
    def init(cls, seed: int, logstd=(0.0, 0.0), out_std: float = 0.01):
        rng = np.random.RandomState(seed)
        flat = np.zeros(P_TOT, np.float32)
        flat[P_W1:P_B1] = normc(rng, (OBD, HID), 1.0).ravel()
        flat[P_W2:P_B2] = normc(rng, (HID, HID), 1.0).ravel()
        flat[P_W3:P_B3] = normc(rng, (HID, ACD), out_std).ravel()
        flat[P_LS:P_TOT] = np.asarray(logstd, np.float32)
        return cls(flat)

    def device_tensors(self, device):
        t = lambda x: torch.as_tensor(np.ascontiguousarray(x, np.float32)).to(device)  # noqa: E731
        return t(self.flat), t(self.ob_mean), t(self.ob_std)


def synthetic_teacher(seed: int = 1, out_std: float = 1.0) -> MlpPolicyParams:
    """Fixed synthetic teacher: seed 1, logstd = fixture values.

    out_std defaults to 1.0 (not baselines' 0.01) so the fixed teacher's actions have the
    magnitude of a trained Reacher teacher (fixture |mean| ~ 0.1-0.5) rather than ~0.01."""
    return MlpPolicyParams.init(seed, logstd=TEACHER_LOGSTD, out_std=out_std)


def student_init(seed: int = 2) -> MlpPolicyParams:
    return MlpPolicyParams.init(seed, logstd=(0.0, 0.0), out_std=0.01)


class TeacherAgent:
    """Mirror of reference teacher.py:12-20: holds ``pi`` (the MlpPolicy parameters).

    ``restore`` with a path loads either the reference's own TF checkpoint (``path`` is the
    Saver prefix, e.g. ".../teacher.ckpt" with its ``.index`` / ``.data-*`` files:
    tf_checkpoint.load_teacher) or a ``.safetensors`` file with the flat params + filter;
    otherwise the synthetic teacher is used."""

    def __init__(self, env=None, sess=None, restore=False, batch=1, seed: int = 1, path: str | None = None):
        if restore and path:
            from . import tf_checkpoint
            if tf_checkpoint.exists(path):
                self.pi = tf_checkpoint.load_teacher(path)
            else:
                from safetensors.numpy import load_file
                d = load_file(path)
                self.pi = MlpPolicyParams(d["flat"].astype(np.float32), d["ob_mean"], d["ob_std"])
        else:
            self.pi = synthetic_teacher(seed)
        self.batch = batch


def save_policy(path: str, p: MlpPolicyParams):
    from safetensors.numpy import save_file
    save_file(dict(flat=p.flat, ob_mean=p.ob_mean, ob_std=p.ob_std), path)


def student_mlp_graph_params(seed: int = 2, in_dim: int = OBD + PDFLAT_SHAPE + 1):
    """Parameters of the reference's student_mlp_graph (student_nn.py:51-57) with TF's
    glorot_uniform kernels and zero biases: [(W, b)] for 16-24-128-128-32-4."""
    rng = np.random.RandomState(seed)
    dims = [in_dim, 24, 128, 128, 32, PDFLAT_SHAPE]
    out = []
    for a, b in zip(dims[:-1], dims[1:]):
        lim = np.sqrt(6.0 / (a + b))
        out.append((rng.uniform(-lim, lim, (a, b)).astype(np.float32), np.zeros(b, np.float32)))
    return out

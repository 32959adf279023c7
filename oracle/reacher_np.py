"""ORACLE (test infrastructure only) -- numpy restatement of Reacher-v2 on MuJoCo 1.50.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this
module, and only as the checker.  The product path (reacherdistilation_amd) never does.

What it restates (the reference's env is third-party, not vendored; pins:
gym==0.10.5, mujoco-py==1.50.1.56 at reference src/distilation/requirement.txt:20,33):
  * gym ReacherEnv.step / reset_model / _get_obs (called from reference
    mlp_train.py:112,135,138,196,200 and lstm_train.py:111,133,136,192,196)
  * MuJoCo 1.50 mj_step with the RK4 integrator (mj_RungeKutta, tableau
    A={.5;0,.5;0,0,1}, B={1/6,1/3,1/3,1/6}) for gym's reacher.xml, two substeps per
    env.step (frame_skip=2), including the joint-1 limit soft constraint and the
    stale-kinematics fingertip (xpos is the last RK stage's, not the final state's).
  * gym seeding (gym/utils/seeding.py: sha512(str(seed))[:8] -> uint32 LE words ->
    RandomState(init_by_array)) and the reset draw order.
  * TimeLimit(max_episode_steps=50).

Parity status: PINNED by the reference's own fixture
(src/distilation/tests/data/dataset.json -> tests/golden/reacher_fixture.npz):
per-step transitions to ~1e-15 (f64), all 25 seed-0 resets bit-exact, all rewards
bit-exact.  See tests/test_oracle_fixture.py.

Derivation of the constants: SURVEY.md Appendix A.
"""
from __future__ import annotations

import hashlib
import struct

import numpy as np

# ---------------------------------------------------------------- model constants
RHO = 1000.0
R_LINK = 0.01          # capsule radius (link0, link1)
L_LINK = 0.1           # capsule half-length*2 (fromto length)
R_TIP = 0.01           # fingertip sphere radius
H_CAP = L_LINK + R_LINK  # MuJoCo 1.50 capsule inertia == cylinder of height L+r


def _inertia_constants():
    m_l = RHO * np.pi * R_LINK ** 2 * H_CAP
    i_c = m_l * (3 * R_LINK ** 2 + H_CAP ** 2) / 12.0
    m_f = RHO * 4.0 / 3.0 * np.pi * R_TIP ** 3
    i_f = 0.4 * m_f * R_TIP ** 2
    a0 = i_c + m_l * 0.05 ** 2 + (m_l + m_f) * 0.1 ** 2
    i2 = i_c + m_l * 0.05 ** 2 + i_f + m_f * 0.11 ** 2
    hc = 0.1 * (m_l * 0.05 + m_f * 0.11)
    return a0, i2, hc


A0, I2, HC = _inertia_constants()
ARMATURE = 1.0
DAMPING = 1.0
GEAR = 200.0
DT = 0.01              # MuJoCo timestep; env.step = FRAME_SKIP substeps
FRAME_SKIP = 2
EPISODE_STEPS = 50     # gym TimeLimit for Reacher-v2 (== reference config.py:17)
LIMIT = 3.0            # joint1 range (-3, 3)
# solref=(0.02,1) solimp=(0.9,0.95,0.001) MuJoCo 1.50 defaults
DMIN, DMAX, WIDTH = 0.9, 0.95, 0.001
TIMECONST = 0.02
B_REF = 2.0 / (DMAX * TIMECONST)
K_REF = 1.0 / (DMAX * DMAX * TIMECONST * TIMECONST)


def _invweight0():
    # (M^-1)_11 at q = 0 (MuJoCo's dof_invweight0 for joint1; it enters R, not A)
    m11 = A0 + I2 + 2 * HC + ARMATURE
    m12 = I2 + HC
    m22 = I2 + ARMATURE
    return m11 / (m11 * m22 - m12 * m12)


INVWEIGHT0 = _invweight0()


# ---------------------------------------------------------------- dynamics
def qacc(q1, v0, v1, ctrl0, ctrl1):
    """Constrained joint accelerations of the 2-link arm (one MuJoCo forward pass).

    Works elementwise on numpy arrays of any float dtype.
    """
    c = np.cos(q1)
    s = np.sin(q1)
    m11 = A0 + I2 + 2 * HC * c + ARMATURE
    m12 = I2 + HC * c
    m22 = I2 + ARMATURE
    # RNE bias (Coriolis/centrifugal), passive damping, actuation (gear 200, ctrlrange +-1)
    b0 = -HC * s * (2 * v0 * v1 + v1 * v1)
    b1 = HC * s * v0 * v0
    t0 = GEAR * np.clip(ctrl0, -1.0, 1.0) - DAMPING * v0 - b0
    t1 = GEAR * np.clip(ctrl1, -1.0, 1.0) - DAMPING * v1 - b1
    det = m11 * m22 - m12 * m12
    i11 = m22 / det
    i12 = -m12 / det
    i22 = m11 / det
    a0 = i11 * t0 + i12 * t1
    a1 = i12 * t0 + i22 * t1
    # joint-1 limit: one scalar soft constraint, solved exactly
    lower = q1 + LIMIT
    upper = LIMIT - q1
    active_lo = lower < 0
    active_hi = upper < 0
    active = active_lo | active_hi
    dist = np.where(active_lo, lower, upper)
    J = np.where(active_lo, 1.0, -1.0)
    x = np.minimum(np.abs(dist) / WIDTH, 1.0)
    y = np.where(x <= 0.5, 2 * x * x, 1 - 2 * (1 - x) * (1 - x))
    d = DMIN + y * (DMAX - DMIN)
    aref = -B_REF * (J * v1) - K_REF * d * dist
    R = (1 - d) / d * INVWEIGHT0
    A = i22
    f = np.maximum(0.0, (aref - J * a1) / (A + R))
    f = np.where(active, f, 0.0)
    a0 = a0 + i12 * J * f
    a1 = a1 + i22 * J * f
    return a0, a1


def fingertip(q0, q1):
    return (0.1 * np.cos(q0) + 0.11 * np.cos(q0 + q1),
            0.1 * np.sin(q0) + 0.11 * np.sin(q0 + q1))


def rk4_substep(q0, q1, v0, v1, c0, c1, h=DT):
    """One mj_step with mjINT_RK4.  Returns new state and the stage-4 position (the
    position MuJoCo's xpos is left at)."""
    k1a0, k1a1 = qacc(q1, v0, v1, c0, c1)
    # stage 2: X0 + h*0.5*F0
    q0b = q0 + h * (0.5 * v0); q1b = q1 + h * (0.5 * v1)
    v0b = v0 + h * (0.5 * k1a0); v1b = v1 + h * (0.5 * k1a1)
    k2a0, k2a1 = qacc(q1b, v0b, v1b, c0, c1)
    # stage 3: X0 + h*0.5*F1
    q0c = q0 + h * (0.5 * v0b); q1c = q1 + h * (0.5 * v1b)
    v0c = v0 + h * (0.5 * k2a0); v1c = v1 + h * (0.5 * k2a1)
    k3a0, k3a1 = qacc(q1c, v0c, v1c, c0, c1)
    # stage 4: X0 + h*F2
    q0d = q0 + h * v0c; q1d = q1 + h * v1c
    v0d = v0 + h * k3a0; v1d = v1 + h * k3a1
    k4a0, k4a1 = qacc(q1d, v0d, v1d, c0, c1)
    b1, b2 = 1.0 / 6.0, 1.0 / 3.0
    dq0 = v0 * b1 + v0b * b2 + v0c * b2 + v0d * b1
    dq1 = v1 * b1 + v1b * b2 + v1c * b2 + v1d * b1
    dv0 = k1a0 * b1 + k2a0 * b2 + k3a0 * b2 + k4a0 * b1
    dv1 = k1a1 * b1 + k2a1 * b2 + k3a1 * b2 + k4a1 * b1
    return (q0 + h * dq0, q1 + h * dq1, v0 + h * dv0, v1 + h * dv1, q0d, q1d)


def observe(q0, q1, v0, v1, tx, ty, kq0, kq1):
    """gym ReacherEnv._get_obs; (kq0,kq1) = the position the kinematics (xpos) is at."""
    fx, fy = fingertip(kq0, kq1)
    z = np.zeros_like(q0)
    return np.stack([np.cos(q0), np.cos(q1), np.sin(q0), np.sin(q1), tx, ty, v0, v1,
                     fx - tx, fy - ty, z], axis=-1)


def reward(tip_dx, tip_dy, a0, a1):
    """ReacherEnv.step: -||fingertip - target|| (f64, stale xpos) - float32(sum float32(a)^2)."""
    a = np.stack([np.asarray(a0, np.float32), np.asarray(a1, np.float32)], axis=-1)
    ctrl = np.square(a).sum(axis=-1)                       # float32, like gym
    dist = np.sqrt(tip_dx * tip_dx + tip_dy * tip_dy)       # np.linalg.norm of [dx,dy,0]
    return -dist - ctrl


# ---------------------------------------------------------------- gym seeding
def gym_seed_words(seed: int) -> list[int]:
    """gym.utils.seeding: _int_list_from_bigint(hash_seed(create_seed(seed)))."""
    seed = seed % 2 ** 64
    digest = hashlib.sha512(str(seed).encode("utf8")).digest()[:8]
    digest += b"\0" * 4                                   # _bigint_from_bytes padding
    words = struct.unpack("3I", digest)
    big = sum(w << (32 * i) for i, w in enumerate(words))
    if big == 0:
        return [0]
    out = []
    while big > 0:
        big, mod = divmod(big, 2 ** 32)
        out.append(mod)
    return out


def gym_rng(seed: int) -> np.random.RandomState:
    rng = np.random.RandomState()
    rng.seed(gym_seed_words(seed))
    return rng


def reset_draw(rng: np.random.RandomState):
    """ReacherEnv.reset_model draw order; returns (q0,q1,v0,v1,tx,ty)."""
    qpos = rng.uniform(low=-0.1, high=0.1, size=4)        # + init_qpos (arm: 0)
    while True:
        goal = rng.uniform(low=-0.2, high=0.2, size=2)
        if np.linalg.norm(goal) < 2:
            break
    qvel = rng.uniform(low=-0.005, high=0.005, size=4)
    return qpos[0], qpos[1], qvel[0], qvel[1], goal[0], goal[1]


class ReacherOracle:
    """Single-env gym-shaped Reacher-v2 (f64 by default); the checker for the HIP env."""

    def __init__(self, seed: int = 0, dtype=np.float64):
        self.dtype = dtype
        self.rng = gym_rng(seed)
        self.elapsed = 0
        self.state = None

    def set_state(self, q0, q1, v0, v1, tx, ty):
        d = self.dtype
        self.state = [d(q0), d(q1), d(v0), d(v1), d(tx), d(ty)]
        self.kin = (self.state[0], self.state[1])   # set_state -> sim.forward(): fresh
        self.elapsed = 0

    def reset(self):
        self.set_state(*reset_draw(self.rng))
        return self.obs()

    def obs(self):
        q0, q1, v0, v1, tx, ty = self.state
        return observe(q0, q1, v0, v1, tx, ty, *self.kin)

    def step(self, a):
        a = np.asarray(a, dtype=np.float32).reshape(-1)
        ob = self.obs()
        r = reward(ob[8], ob[9], a[0], a[1])
        q0, q1, v0, v1, tx, ty = self.state
        c0 = self.dtype(a[0]); c1 = self.dtype(a[1])
        for _ in range(FRAME_SKIP):
            q0, q1, v0, v1, kq0, kq1 = rk4_substep(q0, q1, v0, v1, c0, c1)
        self.state = [q0, q1, v0, v1, tx, ty]
        self.kin = (kq0, kq1)
        self.elapsed += 1
        done = self.elapsed >= EPISODE_STEPS
        return self.obs(), float(r), done, dict(reward_dist=float(-np.hypot(ob[8], ob[9])),
                                                 reward_ctrl=float(-np.square(a).sum()))

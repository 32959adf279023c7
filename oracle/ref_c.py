"""ORACLE (test infrastructure only): ctypes binding of oracle/_build/libreacher_oracle.so.

Importable only from tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "_build", "libreacher_oracle.so")
_lib = None

P = ctypes.c_void_p
I64 = ctypes.c_int64


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_SO):
            build()
        L = ctypes.CDLL(_SO)
        for nm in ("rdo_step_f64", "rdo_step_f32"):
            getattr(L, nm).argtypes = [I64, P, P, P, P]
        for nm in ("rdo_reset_f64", "rdo_reset_f32"):
            getattr(L, nm).argtypes = [I64, P, P, P]
        L.rdo_philox_draw.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32, P]
        L.rdo_philox_reset.argtypes = [I64, I64, ctypes.c_uint64, ctypes.c_uint32, P]
        L.rdo_distill_step.argtypes = [I64, I64, I64, ctypes.c_uint64, I64, P, P, P, P, P, P, P,
                                       ctypes.c_int, ctypes.c_int, ctypes.c_int, P, P, ctypes.c_int]
        L.rdo_adam_tf1.argtypes = [I64, P, P, P, P, ctypes.c_float, ctypes.c_float, ctypes.c_float,
                                   ctypes.c_float, ctypes.c_float, ctypes.c_float]
        L.rdo_constants.argtypes = [P]
        L.rdo_param_count.restype = ctypes.c_int
        _lib = L
    return _lib


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def step(state, act, dtype=np.float64):
    """state [8,n] (modified in place), act [n,2] float32 -> (obs [n,11], rew [n])."""
    n = state.shape[1]
    assert state.dtype == dtype and state.flags.c_contiguous
    act = np.ascontiguousarray(act, dtype=np.float32)
    obs = np.zeros((n, 11), dtype)
    rew = np.zeros(n, dtype)
    fn = lib().rdo_step_f64 if dtype == np.float64 else lib().rdo_step_f32
    fn(n, _p(state), _p(act), _p(obs), _p(rew))
    return obs, rew


def reset(draws, dtype=np.float64):
    """draws [n,6] (q0,q1,v0,v1,tx,ty) -> (state [8,n], obs [n,11])."""
    draws = np.ascontiguousarray(draws, dtype=dtype)
    n = draws.shape[0]
    state = np.zeros((8, n), dtype)
    obs = np.zeros((n, 11), dtype)
    fn = lib().rdo_reset_f64 if dtype == np.float64 else lib().rdo_reset_f32
    fn(n, _p(state), _p(draws), _p(obs))
    return state, obs


def philox_draws(seed, env_ids, episode):
    out = np.zeros((len(env_ids), 6), np.float32)
    L = lib()
    for j, e in enumerate(env_ids):
        L.rdo_philox_draw(seed, int(e), episode, _p(out[j]))
    return out


def philox_reset(n, env_base, seed, episode=0):
    state = np.zeros((8, n), np.float32)
    lib().rdo_philox_reset(n, env_base, seed, episode, _p(state))
    return state


def param_count():
    return lib().rdo_param_count()


def distill_step(state, step, teacher, student, *, seed=0, loss="mse", act_student=False,
                 n_global=None, env_base=0, stagger=False, nthreads=1):
    """One rollout+distill step (f32, CPU).  teacher/student = (params, obmu, obsd).
    Returns (grad [P] f32, metrics [4] f64).  state modified in place."""
    n = state.shape[1]
    grad = np.zeros(param_count(), np.float32)
    met = np.zeros(4, np.float64)
    tp, tmu, tsd = [np.ascontiguousarray(x, np.float32) for x in teacher]
    sp, smu, ssd = [np.ascontiguousarray(x, np.float32) for x in student]
    lib().rdo_distill_step(n, n_global or n, env_base, seed, step, _p(state), _p(tp), _p(tmu),
                           _p(tsd), _p(sp), _p(smu), _p(ssd), 0 if loss == "mse" else 1,
                           1 if act_student else 0, 1 if stagger else 0, _p(grad), _p(met), nthreads)
    return grad, met


def adam_tf1(theta, m, v, g, b1p, b2p, lr=1e-4, b1=0.9, b2=0.999, eps=1e-8):
    """One TF1 ApplyAdam; b1p/b2p = float32 beta powers of this step (b1**t, b2**t)."""
    lib().rdo_adam_tf1(theta.size, _p(theta), _p(m), _p(v), _p(np.ascontiguousarray(g, np.float32)),
                       b1p, b2p, lr, b1, b2, eps)

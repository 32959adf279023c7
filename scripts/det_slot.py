"""Diagnostic (libreacher_dbgslot.so, -DRD_DEBUG_SLOT): with the consumer-side env step, count
slot-tag mismatches (ctl[9]), slot-vs-act-row mismatches (ctl[10]) and lanes that never took
their action (ctl[11]) over a few rollouts.  RD_LIB=libreacher_dbgslot.so RDD_PHYS=consumer."""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from reacherdistilation_amd import _native as nat  # noqa: E402
from reacherdistilation_amd.distill import DistillConfig, DistillTrainer  # noqa: E402

lib = nat.load()
lib.rdd_debug_ctl.restype = ctypes.c_int
lib.rdd_debug_ctl.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
for name, kw in (("c4 split", dict(n_envs=262144, f32_split=True)), ("c4 exact", dict(n_envs=262144)),
                 ("c5", dict(n_envs=131072, act_with="student", student_dtype="bf16", f32_split=True))):
    ref = None
    for rep in range(4):
        tr = DistillTrainer(DistillConfig(seed=5, **kw), device="cuda:0")
        tr.rollout()
        c = np.zeros(16, np.uint32)
        lib.rdd_debug_ctl(tr._h, c.ctypes.data_as(ctypes.c_void_p))
        st = tr.env_state().cpu().numpy()
        if ref is None:
            ref = st
        bad = np.flatnonzero((st != ref).any(0))
        print(name, rep, "tag mismatches", c[9], "slot/act-row mismatches", c[10], "no-action lanes", c[11],
              "state-vs-obs mismatches", c[13], "timeout", c[8], "envs differing from run 0", len(bad),
              (bad[:3] % 64).tolist())
        tr.close()

#!/usr/bin/env python3
"""Generate tests/golden/reacher_fixture.npz from the reference's own test fixture.

Input (read once, here, never on the GPU box):
    /root/reference/src/distilation/tests/data/dataset.json
    -- gzip'd JSON written by json_tricks.dumps(compression=True, primitives=True)
       (reference dataset.py:31-35).  25 episodes x 50 step records, keys
       ob[11], rew, t[4], s[4], with, prev[4] (reference dataset.py:118-143).

Output: plain arrays only (this is data, not code):
    ob    [E,50,11] f64   observation handed to the policy at each step
    act   [E,50,2]  f64   action applied to env.step (t[:2] if with=='t' else s[:2]);
                          float32-representable values
    rew   [E,50]    f64   the record's `rew` = reward of the PREVIOUS env.step
                          (reference mlp_train.py:127-135 writes the reward before stepping)
    t     [E,50,4]  f64   teacher pdflat (mean|logstd)
    s     [E,50,4]  f64   student pdflat (zeros for teacher-stepped records)
    student [E,50]  bool  with=='s'
    prev  [E,50,4]  f64   stored `prev` pdflat
The loader is json + gzip from the standard library: nothing in the file is executed.
"""
import gzip
import json
import os
import sys

import numpy as np

REF = "/root/reference/src/distilation/tests/data/dataset.json"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "reacher_fixture.npz")


def main(src=REF, out=OUT):
    with open(src, "rb") as fh:
        episodes = json.loads(gzip.decompress(fh.read()))
    E = len(episodes)
    T = len(episodes[0])
    assert all(len(e) == T for e in episodes)
    ob = np.zeros((E, T, 11))
    act = np.zeros((E, T, 2))
    rew = np.zeros((E, T))
    t = np.zeros((E, T, 4))
    s = np.zeros((E, T, 4))
    stu = np.zeros((E, T), dtype=bool)
    prev = np.zeros((E, T, 4))
    for e, ep in enumerate(episodes):
        for k, rec in enumerate(ep):
            ob[e, k] = rec["ob"]
            r = rec["rew"]
            rew[e, k] = r[0] if isinstance(r, list) else r
            t[e, k] = rec["t"]
            s[e, k] = rec["s"]
            stu[e, k] = rec["with"] == "s"
            prev[e, k] = rec["prev"]
            act[e, k] = (s if stu[e, k] else t)[e, k, :2]
    # actions are float32 values (TF outputs); check so the golden is what the env saw
    assert np.array_equal(act.astype(np.float32).astype(np.float64), act)
    np.savez_compressed(out, ob=ob, act=act, rew=rew, t=t, s=s, student=stu, prev=prev)
    print(f"wrote {out}: {E} episodes x {T} steps")


if __name__ == "__main__":
    main(*sys.argv[1:])

"""PPO teacher training throughput (csrc/ppo.hip): env steps per second of whole iterations
(rollout + GAE + filter + 10 epochs of minibatch Adam), and the learning curve."""
import json
import sys
import time

import torch

sys.path.insert(0, ".")
from reacherdistilation_amd.ppo import METRICS, PPOConfig, PPOTrainer  # noqa: E402


def cpu_baseline(n=64, T=50, mb=64, seconds=4.0):
    """The oracle (numpy f64 policy/value math + the C f64 env, one core) doing PPO: an
    actor batch of n envs x T steps, GAE, and minibatch gradient steps (the reference's
    minibatch 64, 10 epochs), timed per env step of whole iterations."""
    import threadpoolctl
    import numpy as np

    from oracle import policy_np as pn
    from oracle import ppo_np as pp
    from oracle import ref_c
    rs = np.random.RandomState(0)
    pol = np.concatenate([pn.normc(rs, (11, 64), 1.0).ravel(), np.zeros(64), pn.normc(rs, (64, 64), 1.0).ravel(),
                          np.zeros(64), pn.normc(rs, (64, 2), 0.01).ravel(), np.zeros(2), np.zeros(2)])
    vf = np.concatenate([pn.normc(rs, (11, 64), 1.0).ravel(), np.zeros(64), pn.normc(rs, (64, 64), 1.0).ravel(),
                         np.zeros(64), pn.normc(rs, (64, 1), 1.0).ravel(), np.zeros(1)])
    opt = pn.AdamTF1(pp.P_POL + pp.P_VF, lr=3e-4, dtype=np.float64)
    with threadpoolctl.threadpool_limits(1):
        t0, iters = time.perf_counter(), 0
        while time.perf_counter() - t0 < seconds:
            state = ref_c.philox_reset(n, 0, 0, iters).astype(np.float64)
            obs, acs, vps, rws = [], [], [], []
            ob, _ = ref_c.step(state.copy(), np.zeros((n, 2), np.float32), np.float64)
            for _t in range(T):
                z = pp.obz(ob, 0.0, 1.0)
                fp, fv = pp.pol_forward(pol, z), pp.vf_forward(vf, z)
                a = (fp["mean"] + np.exp(fp["logstd"]) * rs.randn(n, 2)).astype(np.float32)
                obs.append(ob); acs.append(a); vps.append(fv["v"])
                ob, r = ref_c.step(state, a, np.float64)
                rws.append(r)
            adv, ret = pp.gae(np.array(rws), np.array(vps), np.zeros((T, n)), np.zeros(n))
            Z = pp.obz(np.concatenate(obs), 0.0, 1.0)
            A = np.concatenate(acs).astype(np.float64)
            fp = pp.pol_forward(pol, Z)
            lpo = pp.logp(fp["mean"], fp["logstd"], A)
            atarg = pp.standardize(adv.ravel())
            for _epoch in range(10):                       # optim_epochs
                idx = rs.permutation(n * T)
                for b in range(0, n * T - mb + 1, mb):
                    i = idx[b:b + mb]
                    r_ = pp.loss_and_grads(pol, vf, Z[i], A[i], lpo[i], atarg[i], ret.ravel()[i], 0.2)
                    x = opt.step(np.concatenate([pol, vf]), np.concatenate([r_["gpol"], r_["gvf"]]))
                    pol, vf = x[:pp.P_POL], x[pp.P_POL:]
            iters += 1
        el = time.perf_counter() - t0
    return {"cpu_env_steps_per_s": n * T * iters / el, "cpu_iterations": iters, "cpu_actor_batch": n * T, "cpu_minibatch": mb,
            "cpu_cores": 1, "cpu_kind": "oracle/ppo_np.py + C f64 env (numpy f64)"}


def main():
    n, T, mb, iters = 4096, 50, 4096, 40
    if "--mb" in sys.argv:                                 # e.g. --mb 64: the reference's minibatch
        mb = int(sys.argv[sys.argv.index("--mb") + 1])
    if "--iters" in sys.argv:
        iters = int(sys.argv[sys.argv.index("--iters") + 1])
    tr = PPOTrainer(PPOConfig(n_envs=n, horizon=T, optim_batchsize=mb, max_timesteps=n * T * iters), device="cuda:0")
    tr.iterate()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters - 1):
        tr.iterate()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    m = tr.metrics(iters)
    print(json.dumps({"n_envs": n, "horizon": T, "minibatch": mb, "iter_ms": dt * 1e3 / (iters - 1),
                      "env_steps_per_s": n * T * (iters - 1) / dt,
                      "ep_ret_mean_first": m[0, 0], "ep_ret_mean_last": m[-1, 0],
                      "curve": [round(float(x), 3) for x in m[:, 0]]}), flush=True)
    print(json.dumps(dict(zip(METRICS, map(float, m[-1])))), flush=True)
    if "--no-cpu" not in sys.argv:
        print(json.dumps(cpu_baseline()), flush=True)


if __name__ == "__main__":
    main()

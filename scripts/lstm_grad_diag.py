import sys, os, numpy as np, torch
sys.path.insert(0, os.getcwd())
sys.path.insert(0, os.path.join(os.getcwd(), "tests"))
from test_student_lstm_gpu import _trainer, _batch, _t
from oracle import lstm_np as ln
T, B = 10, 20
ob, prev, t = _batch(T, B, 3 + B)
out = {}
for mode in ("1", "0"):
    tr = _trainer(T, B, "kl", step_recurrence=mode == "0")
    p = tr.params().cpu().numpy()
    out[mode] = tr.rollout(_t(ob), _t(prev), _t(t)).cpu().numpy().astype(np.float64)
    tr.close()
fw = ln.forward(p, ob, prev)
L, d, sq = ln.loss_and_dout(fw["pdflat"], t, "kl", T * B)
want = ln.backward(p, fw, d)
lay = ln.layout(T)[0]
print(list(lay.keys())[:12])
for k, (o, s) in list(lay.items())[:8]:
    n = int(np.prod(s))
    for mode in ("1", "0"):
        g = out[mode][o:o + n]; w = want[o:o + n]
        print(k, s, mode, "rel", float(np.linalg.norm(g - w) / (np.linalg.norm(w) + 1e-30)), "max", float(np.abs(g - w).max()))

"""Command line of the reference's main.py (src/distilation/main.py:9-27):

  python -m reacherdistilation_amd -lt [-k KEEP] [-r]   LSTM distillation (lstm_train.train)
  python -m reacherdistilation_amd -ct [-r]             MLP distillation (mlp_train.train, the
                                                        reference's student_mlp_graph)
  python -m reacherdistilation_amd -ch [-k KEEP]        print the LSTM checkpoint's tensors

Paths as the reference's config.py:40-45 and teacher.py:20, under ``--data-dir`` (default
~/reacher/data): the LSTM checkpoint ``lstm_with_keep_probability_{KEEP}.ckpt`` (a TF
checkpoint, tf_checkpoint), the teacher ``teacher.ckpt`` (restored when present, else the
synthetic teacher, with a message) and the run's dataset pages
``<date>/<time>/{lstm,mlp}/dataset_kp_{KEEP}/``.  Both drivers train with the keep
probability (``-k``, default config KEEP_PROB; lstm_train.py:150, mlp_train.py:151).  Fixed here:
``-k`` reaches the LSTM driver (the reference's ``global KEEP_PROB`` in main.py:17-19 never
does), and ``-ch`` prints the tensors (main.py:23 calls an undefined ``chkp``).  Added:
``--episodes``, ``--warmup``, ``--device``, ``--data-dir``.
"""
from __future__ import annotations

import argparse
import datetime
import os
import sys

import numpy as np

from .config import KEEP_PROB, MLP_EPISODE_BUDGET, TOTAL_EPISODES


def paths(data_dir: str, keep: float, stamp: str | None = None) -> dict:
    """config.py:14-15,36-45 and mlp_train.py:101-106: the dataset pages of a run go to a new
    <date>/<time>/{lstm,mlp}/dataset_kp_<keep> directory."""
    stamp = stamp or datetime.datetime.now().strftime("%Y%m%d/%H%M%S")
    run = os.path.join(data_dir, *stamp.split("/"))
    return {"lstm": os.path.join(data_dir, f"lstm_with_keep_probability_{keep}.ckpt"),
            "teacher": os.path.join(data_dir, "teacher.ckpt"),
            "dataset_lstm": os.path.join(run, "lstm", f"dataset_kp_{keep}"),
            "dataset_mlp": os.path.join(run, "mlp", f"dataset_kp_{keep}")}


def print_tensors(prefix: str, out=print) -> None:
    """inspect_checkpoint.print_tensors_in_checkpoint_file(all_tensors=True,
    all_tensor_names=True): every tensor's name and value, names in order."""
    from . import tf_checkpoint
    t = tf_checkpoint.read(prefix)
    with np.printoptions(threshold=sys.maxsize):
        for name in sorted(t):
            out(f"tensor_name:  {name}")
            out(str(t[name]))


def main(argv=None, log=print) -> int:
    ap = argparse.ArgumentParser(prog="python -m reacherdistilation_amd")
    ap.add_argument("-lt", "--lstm_train", help="train lstm", action="store_true")
    ap.add_argument("-ct", "--mlp_train", help="train mlp", action="store_true")
    ap.add_argument("-k", "--keep_prob", help="keep_prob on lstm ob dropout", nargs=1, type=float, default=None)
    ap.add_argument("-ch", "--check", help="check point", action="store_true")
    ap.add_argument("-r", "--restore", help="restore", action="store_true")
    ap.add_argument("--episodes", type=int, default=None, help="episode budget (default: the driver's)")
    ap.add_argument("--warmup", type=int, default=None, help="teacher-stepped episodes first (default: the driver's)")
    ap.add_argument("--device", default="cuda:0")
    ap.add_argument("--data-dir", default=os.path.join(os.path.expanduser("~"), "reacher", "data"))
    args = ap.parse_args(argv)
    keep = args.keep_prob[0] if args.keep_prob else KEEP_PROB
    p = paths(args.data_dir, keep)
    if args.check:
        log(" checking saved variables ")
        print_tensors(p["lstm"], log)
        return 0
    if not (args.lstm_train or args.mlp_train):
        return 0   # as the reference: no flag, nothing to do
    from . import tf_checkpoint
    teacher = p["teacher"] if tf_checkpoint.exists(p["teacher"]) else None
    if teacher is None:
        log(f"teacher checkpoint {p['teacher']} not found: using the synthetic teacher")
    extra = {} if args.warmup is None else {"warmup_episodes": args.warmup}
    if args.lstm_train:
        from . import lstm_train
        lstm_train.train(True, args.restore, episodes=args.episodes or TOTAL_EPISODES, keep_prob=keep,
                         device=args.device, teacher_path=teacher, student_path=p["lstm"],
                         store_dir=p["dataset_lstm"], log=log, **extra)
    else:
        from . import mlp_train
        mlp_train.train(True, args.restore, episodes=args.episodes or MLP_EPISODE_BUDGET, keep_prob=keep,
                        device=args.device, teacher_path=teacher, student="mlp", store_dir=p["dataset_mlp"],
                        log=log, **extra)
    return 0


if __name__ == "__main__":
    sys.exit(main())

"""The reference main.py's command line (python -m reacherdistilation_amd): flags, paths and
the -ch checkpoint print, on the CPU (the training flags run in tests/test_cli_gpu.py)."""
import numpy as np

from reacherdistilation_amd import __main__ as cli
from reacherdistilation_amd import tf_checkpoint as tc


def test_paths_follow_the_reference_config():
    p = cli.paths("/d", 0.5, "20261017/120000")   # config.py:14-15,36-45, teacher.py:20, mlp_train.py:101-106
    assert p["lstm"] == "/d/lstm_with_keep_probability_0.5.ckpt" and p["teacher"] == "/d/teacher.ckpt"
    assert p["dataset_lstm"] == "/d/20261017/120000/lstm/dataset_kp_0.5"
    assert p["dataset_mlp"] == "/d/20261017/120000/mlp/dataset_kp_0.5"


def test_check_prints_every_tensor(tmp_path):
    tc.write(str(tmp_path / "lstm_with_keep_probability_0.7.ckpt"),
             {"LSTM/dense/bias": np.arange(3, dtype=np.float32), "LSTM/a": np.ones((2, 2), np.float32)})
    out = []
    assert cli.main(["-ch", "-k", "0.7", "--data-dir", str(tmp_path)], log=out.append) == 0
    names = [x for x in out if x.startswith("tensor_name:")]
    assert names == ["tensor_name:  LSTM/a", "tensor_name:  LSTM/dense/bias"]
    assert "[0. 1. 2.]" in out


def test_no_flag_does_nothing():
    assert cli.main([], log=lambda *a: None) == 0

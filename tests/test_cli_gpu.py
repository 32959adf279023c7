"""python -m reacherdistilation_amd -lt / -ct (reference main.py:25-27): both drivers run from
the command line with the reference's paths; -k reaches the LSTM driver; -r restores the LSTM
checkpoint the previous run saved."""
import os

import pytest

pytestmark = pytest.mark.gpu


def test_lstm_and_mlp_training_from_the_command_line(tmp_path):
    from reacherdistilation_amd import __main__ as cli
    from reacherdistilation_amd import tf_checkpoint as tc
    d = str(tmp_path)
    log = []
    assert cli.main(["-lt", "-k", "0.5", "--episodes", "4", "--warmup", "2", "--data-dir", d], log=log.append) == 0
    ck = os.path.join(d, "lstm_with_keep_probability_0.5.ckpt")
    assert tc.exists(ck) and "LSTM/unique_lstm_cell/kernel/Adam" in tc.read(ck)
    assert any("synthetic teacher" in m for m in log)
    log.clear()
    assert cli.main(["-lt", "-r", "--episodes", "4", "--warmup", "2", "--data-dir", d], log=log.append) == 0
    assert not any("does not exist" in m for m in log)          # restored
    assert cli.main(["-ct", "--episodes", "3", "--warmup", "1", "--data-dir", d], log=log.append) == 0

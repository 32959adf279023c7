"""Constants mirroring the reference's module config (reference src/distilation/config.py:17-32).

Only the shape/loop constants are restated; the reference's import-time directory
creation (config.py:34-48) is deliberately not (it is a side effect, not configuration).
"""
EPISODE_STEPS = 50        # config.py:17  (gym TimeLimit of Reacher-v2)
OBSPACE_SHAPE = 11        # config.py:18
ACSPACE_SHAPE = 2         # config.py:19
PDFLAT_SHAPE = 4          # config.py:20  (mean[2] | logstd[2])
GAMMA = 0.99              # config.py:21
TOTAL_EPISODES = 8000     # config.py:24
STEPS_UNROLLED = 10       # config.py:25
LSTM_BATCH_SIZE = 20      # config.py:26
MLP_BATCH_SIZE = 20       # config.py:28
NUM_UNITS = 200           # config.py:29
KEEP_PROB = 0.5           # config.py:30
MAX_CAPACITY = 10         # config.py:31
TRAINING_EPOCHS = 1       # config.py:32

# Fixture-derived teacher log-std: the reference teacher's state-independent
# logstd, constant in every record of src/distilation/tests/data/dataset.json.
TEACHER_LOGSTD = (-3.2939295768737793, -3.3629262447357178)

# MLP reference step budget: 5000 episodes x 50 steps (mlp_train.py:204)
MLP_EPISODE_BUDGET = 5000

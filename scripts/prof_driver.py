import cProfile, pstats, sys, os, time
sys.path.insert(0, os.getcwd())
import torch
from reacherdistilation_amd import mlp_train
mlp_train.train(episodes=60, log=lambda *a: None)   # warm
torch.cuda.synchronize()
pr = cProfile.Profile()
t0 = time.perf_counter()
pr.enable()
tr, ds, _ = mlp_train.train(episodes=120, log=lambda *a: None)
torch.cuda.synchronize()
pr.disable()
print("seconds", time.perf_counter() - t0, "steps", ds.num_episodes() * 50)
pstats.Stats(pr).sort_stats("tottime").print_stats(25)

"""Reward extraction from dataset pages (reference src/distilation/extract_reward.py:12-48,
247-252): the return of every episode of a run's pages in page order, averaged per
``per_episodes`` episodes, and divided by EPISODE_STEPS for the average per-step reward.

``ExtractReward`` keeps the reference's class methods and arithmetic (Python float sums in
record order, the last group possibly shorter); ``dataset`` is a page directory or a
``pages.PageStore`` (the reference passes its ``Dataset(path)``).  ``device_returns`` is the
same per-episode return over a ``DeviceDataset``'s ring, summed on the device (f32) for
collections too large to page through the host.  ``extract(path, out)`` is the reference
script's loop body: it saves the averages with ``np.save`` and returns them.
"""
from __future__ import annotations

import numpy as np

from .config import EPISODE_STEPS
from .pages import PageStore, read_page


def _pages(dataset) -> list:
    store = dataset if isinstance(dataset, PageStore) else PageStore(str(dataset))
    return store.sorted_pages()   # Dataset.pages(): by page index (dataset.py:87-96)


class ExtractReward:
    @classmethod
    def get_episode_reward(cls, episode) -> list:
        return [float(r["rew"][0]) if isinstance(r["rew"], list) else float(r["rew"]) for r in episode]

    @classmethod
    def get_return(cls, dataset) -> list:
        ret = []
        for page in _pages(dataset):
            for episode in read_page(page):
                ret.append(sum(cls.get_episode_reward(episode)))
        return ret

    @classmethod
    def get_avg_return(cls, dataset, per_episodes: int) -> list:
        ret = cls.get_return(dataset)
        return [sum(ret[i:i + per_episodes]) / len(ret[i:i + per_episodes]) for i in range(0, len(ret), per_episodes)]

    @classmethod
    def get_avg_reward(cls, dataset, per_episodes: int) -> list:
        return [r / EPISODE_STEPS for r in cls.get_avg_return(dataset, per_episodes)]


def device_returns(ds):
    """Return of every episode in a DeviceDataset's ring, oldest first (the rew column summed
    over each episode's records, f32 on the device)."""
    import torch
    from .dataset import F_REW
    n = ds.stored()
    first = ds.num_episodes() - n
    slots = torch.tensor([(first + e) % ds.capacity for e in range(n)], dtype=torch.long, device=ds.device)
    lens = torch.tensor([ds.lens[int(s)] for s in slots.tolist()], device=ds.device)
    rew = ds.ring[slots, :, F_REW]
    mask = torch.arange(EPISODE_STEPS, device=ds.device)[None, :] < lens[:, None]
    return (rew * mask).sum(1)


def extract(path: str, out: str, per_episodes: int = 5, log=print) -> list:
    avg_rews = ExtractReward.get_avg_reward(path, per_episodes)
    log(avg_rews)
    np.save(out, avg_rews)
    log("file written to {0}.npy, avg_rews array length is {1}".format(out, len(avg_rews)))
    return avg_rews

"""Dataset pages in the reference's on-disk format (reference dataset.py:14-65 DatasetStore,
:72-96 Dataset.dump / pages).

A page is what ``json_tricks.dumps(obj=data_in_memory, compression=True, primitives=True)``
writes (dataset.py:31-35): gzip-compressed plain JSON of a list of episodes, each a list of
step records ``{"ob": [11], "rew": r or [r], "t": [4], "s": [4], "with": "t"|"s",
"prev": [4], "prew": [r]}`` (dataset.py:118-143; older pages, like the reference's test
fixture, carry a scalar ``rew`` and no ``prew``).  json_tricks is not needed for this
subset: with ``primitives=True`` numpy arrays are written as plain lists, so the standard
library's json + gzip read and write the same bytes' content.  Loading executes nothing
from the file.

``PageStore`` mirrors DatasetStore (page names ``dataset_<k>.json``, a new page once one
holds MAX_CAPACITY episodes, FileExistsError instead of overwriting); ``DeviceDataset.dump``
/ ``load_page`` move episodes between the device ring and pages.
"""
from __future__ import annotations

import gzip
import json
import os
import random
import re

import numpy as np

from .config import EPISODE_STEPS, MAX_CAPACITY, OBSPACE_SHAPE, PDFLAT_SHAPE

F_OB, F_REW, F_T, F_S, F_WITH = 0, OBSPACE_SHAPE, OBSPACE_SHAPE + 1, OBSPACE_SHAPE + 1 + PDFLAT_SHAPE, \
    OBSPACE_SHAPE + 1 + 2 * PDFLAT_SHAPE
REC = F_WITH + 1


def read_page(path: str) -> list:
    """Episodes of a page (gzip'd or plain JSON)."""
    with open(path, "rb") as fh:
        raw = fh.read()
    if raw[:2] == b"\x1f\x8b":
        raw = gzip.decompress(raw)
    eps = json.loads(raw)
    if not isinstance(eps, list) or not all(isinstance(e, list) for e in eps):
        raise ValueError(f"{path}: not a dataset page (a list of episodes)")
    return eps


def write_page(path: str, episodes: list):
    data = gzip.compress(json.dumps(episodes).encode())
    tmp = path + ".tmp"
    with open(tmp, "wb") as fh:
        fh.write(data)
    os.replace(tmp, path)


def _scalar(v) -> float:
    return float(v[0]) if isinstance(v, (list, tuple)) else float(v)


def episodes_to_records(episodes, with_lengths: bool = False):
    """[E, EPISODE_STEPS, 21] f64 records (ob | rew | t | s | with) of the complete episodes;
    with_lengths=True: of EVERY episode (an incomplete one zero-padded, as the reference's
    flush stores them, dataset.py:146-149), and their lengths [E]."""
    full = [e for e in episodes if len(e) <= EPISODE_STEPS and (with_lengths or len(e) == EPISODE_STEPS)]
    out = np.zeros((len(full), EPISODE_STEPS, REC))
    lens = np.array([len(e) for e in full], np.int64)
    for i, ep in enumerate(full):
        for k, st in enumerate(ep):
            out[i, k, F_OB:F_REW] = st["ob"]
            out[i, k, F_REW] = _scalar(st["rew"])
            out[i, k, F_T:F_S] = st["t"]
            out[i, k, F_S:F_WITH] = st.get("s", [0.0] * PDFLAT_SHAPE)
            out[i, k, F_WITH] = 1.0 if st.get("with", "t") == "s" else 0.0
    return (out, lens) if with_lengths else out


def records_to_episodes(rec, lens=None) -> list:
    """Inverse of episodes_to_records, with the prev / prew fields the reference derives
    (previous record's teacher pdflat and reward, zeros at t = 0; dataset.py:132-133,152-163);
    lens: each episode's record count (default: all EPISODE_STEPS)."""
    rec = np.asarray(rec, np.float64)
    eps = []
    for i, ep in enumerate(rec):
        steps = []
        for k, r in enumerate(ep[:EPISODE_STEPS if lens is None else int(lens[i])]):
            prev = ep[k - 1, F_T:F_S].tolist() if k > 0 else [0.0] * PDFLAT_SHAPE
            prew = [float(ep[k - 1, F_REW])] if k > 0 else [0]
            steps.append({"ob": r[F_OB:F_REW].tolist(), "rew": [float(r[F_REW])], "t": r[F_T:F_S].tolist(),
                          "s": r[F_S:F_WITH].tolist(), "with": "s" if r[F_WITH] > 0.5 else "t",
                          "prev": prev, "prew": prew})
        eps.append(steps)
    return eps


class PageStore:
    """DatasetStore (reference dataset.py:14-65)."""

    def __init__(self, dir_path: str):
        self.dir_path = dir_path
        os.makedirs(dir_path, exist_ok=True)
        self.pages = self.collect_pages(dir_path)
        self.curr_page = self.get_full_path(0)

    def get_full_path(self, page=None) -> str:
        # as the reference: the next page index is the number of finished pages
        return os.path.join(self.dir_path, f"dataset_{len(self.pages)}.json")

    def store(self, data_in_memory: list) -> list:
        write_page(self.curr_page, data_in_memory)
        if len(data_in_memory) >= MAX_CAPACITY:
            self.curr_page = self.create_new_page()
            return []
        return data_in_memory

    def load(self, page: str) -> list:
        return read_page(page)

    def rand_pages(self, num_pages: int):
        if not self.pages:
            return None
        return random.sample(self.pages, min(num_pages, len(self.pages)))

    def create_new_page(self) -> str:
        self.pages.append(self.curr_page)
        page = self.get_full_path(len(self.pages))
        if os.path.exists(page):
            raise FileExistsError("current page already exists. will not overwrite")
        return page

    @staticmethod
    def collect_pages(dir_path: str) -> list:
        return [os.path.join(dir_path, f) for f in os.listdir(dir_path)
                if os.path.isfile(os.path.join(dir_path, f)) and re.fullmatch(r"dataset_\d+\.json", f)]

    def sorted_pages(self) -> list:
        """Dataset.pages() (reference dataset.py:87-96): pages by their index."""
        return sorted(self.pages, key=lambda p: int(re.search(r"dataset_(\d+)\.json", p).group(1)))

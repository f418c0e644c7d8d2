"""Data feed of the training path: the reference's SequenceDataset /
DatasetLoader (processing/dataset.py:57-200, 264-321) with the token store
resident in HBM.

The reference loads one ``<root>/<band>/<song>.npy`` file per sample, cuts the
window on the host and copies it to the GPU (``dataset.py:186,193``). Here
every song is loaded once into one int32 device buffer (a few hundred MB even
for large MIDI corpora, against 288 GB of HBM) and a batch is ONE launch of
``msq_window_gather`` (csrc/data.hip): B windows of T+1 tokens, zero padding,
the optional augmentation, src / trg / metadata written in place. The host
only draws the sampler indices and window starts (the reference's
``WeightedRandomSampler`` and ``random.randint`` semantics) and hands B x 5
int64 parameters to the device.

Same surfaces: ``SequenceDataset(directory)[i] -> (src, trg, meta)``,
``len``, ``file_prob()``; ``DatasetLoader(directory, batch_size, test_ratio)
.get_dataloaders() -> (train, test)`` iterables of device batches;
``get_dataloader_full(shuffle)``. Metadata tokens follow
``get_metadata_dict`` (dataset.py:76-132)."""
import ctypes
import json
import os
import random
from pathlib import Path

import numpy as np
import torch

from ._lib import ptr, call, stream
from .config import BLOCK_LEN, DEFAULT_DISC, N_META, Discretization


def _floor10(x):
    return (x // 10) * 10


def metadata_tokens(metadata: dict):
    """Band -> 6 metadata tokens [band, genre x4 (padded), decade] and the
    tokenization tables, as SequenceDataset.get_metadata_dict
    (dataset.py:76-132) computes them from metadata.json. The reference also
    rewrites tokenization.json as a side effect (:47-52); here the tables are
    returned instead (VOCAB_SIZE = metadata vocabulary size, :49)."""
    genre_list, bands = [], {}
    min_t, max_t = 1e9, 0
    for a in metadata["artists"]:
        dec = _floor10(a["year_started"])
        min_t, max_t = min(min_t, dec), max(max_t, dec)
        for gname in a["genres"]:
            if gname not in genre_list:
                genre_list.append(gname)
        bands[a["name"]] = {"decade": dec, "genres": a["genres"]}
    n_dec = (max_t - min_t) // 10 + 1
    start_dec = 1
    start_genre = start_dec + n_dec + 1
    start_band = start_genre + len(genre_list) + 1
    band_tok = {b: i + start_band for i, b in enumerate(bands)}
    time_tok = {t: i + start_dec for i, t in enumerate(range(int(min_t), int(max_t) + 1, 10))}
    genre_tok = {gname: i + start_genre for i, gname in enumerate(genre_list)}
    tok = {"time_tokenized": dict(time_tok), "genre_tokenized": dict(genre_tok), "band_tokenized": dict(band_tok)}
    tok["time_tokenized"][None] = start_dec - 1
    tok["genre_tokenized"][None] = start_genre - 1
    tok["band_tokenized"][None] = start_band - 1
    tok["VOCAB_SIZE"] = sum(len(v) for k, v in tok.items() if k != "VOCAB_SIZE")
    meta = {}
    for b, e in bands.items():
        gs = [genre_tok[gname] for gname in e["genres"]]
        if len(gs) < 4:
            gs += [start_genre - 1] * (4 - len(gs))
        meta[b] = [band_tok[b]] + gs + [time_tok[e["decade"]]]
    return meta, tok


class SequenceDataset:
    """Device-resident SequenceDataset (dataset.py:57-200).

    directory: ``<root>/<band>/<song>.npy`` int64 1-D token arrays.
    metadata: metadata.json path or its parsed dict (band names = directory names).
    Songs are listed with os.walk and shuffled (dataset.py:66-71) with
    ``shuffle_rng`` (default: ``rng``); ``rng`` draws the window starts and
    augmentation shifts. Under data parallelism the shuffle must be identical
    on every rank (the train/test split and the DistributedSampler shards
    index the shuffled list) while the window draws differ per rank, so
    DatasetLoader passes a rank-independent ``shuffle_rng``."""

    def __init__(self, directory, metadata, block_len=BLOCK_LEN, device="cuda", disc: Discretization = None,
                 augmentation=False, start_of_seq=False, end_of_seq=False, rng: random.Random = None,
                 shuffle_rng: random.Random = None):
        self.directory = directory
        self.sequence_length = block_len
        self.disc = disc or DEFAULT_DISC
        self.augmentation, self.start_of_seq, self.end_of_seq = augmentation, start_of_seq, end_of_seq
        self.rng = rng or random.Random()
        if not isinstance(metadata, dict):
            with open(metadata, "r", encoding="utf-8") as f:
                metadata = json.load(f)
        self.metadata_dict, self.tokenizations = metadata_tokens(metadata)
        self.file_paths = []
        for root, _, files in os.walk(directory):
            for fn in files:
                if fn.endswith(".npy"):
                    self.file_paths.append(os.path.join(root, fn))
        self.num_files = len(self.file_paths)
        (shuffle_rng or self.rng).shuffle(self.file_paths)
        if not self.file_paths:
            raise ValueError(f"no .npy token files under {directory}")
        # one pass over the corpus: lengths, token store, per-song metadata
        arrays = [np.load(p, allow_pickle=False) for p in self.file_paths]
        for p, a in zip(self.file_paths, arrays):
            if a.ndim != 1 or not np.issubdtype(a.dtype, np.integer):
                raise ValueError(f"{p}: expected a 1-D integer token array, got {a.dtype} {a.shape}")
        self.lengths = np.array([len(a) for a in arrays], dtype=np.int64)
        off = np.zeros(len(arrays), dtype=np.int64)
        off[1:] = np.cumsum(self.lengths)[:-1]
        flat = np.concatenate(arrays).astype(np.int32) if self.lengths.sum() else np.zeros(1, np.int32)
        meta = np.array([self.metadata_dict[Path(p).parts[-2]] for p in self.file_paths], dtype=np.int64)
        self.device = torch.device(device)
        self.tokens = torch.from_numpy(flat).to(self.device)
        self.song_off = torch.from_numpy(off).to(self.device)
        self.song_len = torch.from_numpy(self.lengths).to(self.device)
        self.song_meta = torch.from_numpy(meta.reshape(-1, N_META)).to(self.device)
        d = self.disc
        self._disc_arr = (ctypes.c_int64 * 6)(d.pitch, d.channel, d.dyn, d.length, d.time, d.tempo)
        self._disc = ctypes.cast(self._disc_arr, ctypes.c_void_p)  # host array

    def __len__(self):
        return len(self.file_paths)

    def file_prob(self):
        """Sampling weight of each song: its length share (dataset.py:197-200)."""
        return self.lengths / self.lengths.sum()

    def window_params(self, idx):
        """{song, start, note shift, velocity shift, 2 x time factor} of one
        sample, drawing from self.rng in the order __getitem__ does
        (dataset.py:176-188; augmentation draws :136-152)."""
        n, T1 = int(self.lengths[idx]), self.sequence_length + 1
        ix = 0
        if n > T1:
            if self.end_of_seq:
                ix = n - T1 - 1
            elif self.start_of_seq:
                ix = 0
            else:
                ix = self.rng.randint(0, n - T1)
        note = vel = 0
        f2 = 2
        if self.augmentation:
            note = self.rng.randint(-12, 12)
            vel = self.rng.randint(-20, 20)
            f2 = self.rng.randint(1, 8)  # time factor = f2 / 2
        return [int(idx), ix, note, vel, f2]

    def gather(self, params, out=None):
        """One launch: windows of the B parameter rows -> (src, trg, meta) on the device."""
        p = torch.as_tensor(params, dtype=torch.int64)
        if p.device != self.device:
            p = p.pin_memory().to(self.device, non_blocking=True) if self.device.type == "cuda" else p.to(self.device)
        B, T = p.shape[0], self.sequence_length
        if out is None:
            out = (torch.empty(B, T, dtype=torch.int64, device=self.device),
                   torch.empty(B, T, dtype=torch.int64, device=self.device),
                   torch.empty(B, N_META, dtype=torch.int64, device=self.device))
        src, trg, meta = out
        call("msq_window_gather", ptr(src), ptr(trg), ptr(meta), ptr(self.tokens), ptr(self.song_off),
             ptr(self.song_len), ptr(self.song_meta), N_META, ptr(p), B, T, int(self.augmentation),
             self._disc, stream())
        return src, trg, meta

    def __getitem__(self, idx):
        src, trg, meta = self.gather([self.window_params(idx)])
        return src[0], trg[0], meta[0]


class _Subset:
    def __init__(self, dataset, indices):
        self.dataset, self.indices = dataset, list(indices)

    def __len__(self):
        return len(self.indices)


def random_split(dataset, lengths, generator=None):
    """torch.utils.data.random_split of the song indices."""
    perm = torch.randperm(sum(lengths), generator=generator).tolist()
    out, o = [], 0
    for n in lengths:
        out.append(_Subset(dataset, perm[o:o + n]))
        o += n
    return out


class DeviceLoader:
    """DataLoader(subset, batch_size, sampler) equivalent: each epoch draws
    the sampler's indices (weighted with replacement, or a per-rank shuffled
    shard), then yields device batches (src [B,T], trg [B,T], meta [B,6]);
    the last partial batch is kept, as DataLoader's drop_last=False."""

    def __init__(self, subset, batch_size, weights=None, rank=0, world=1, generator=None):
        self.subset, self.batch_size = subset, batch_size
        self.weights = None if weights is None else torch.as_tensor(weights, dtype=torch.float64)
        self.rank, self.world = rank, world
        self.g = generator or torch.Generator()

    def _indices(self):
        idx = self.subset.indices
        if self.weights is not None:  # WeightedRandomSampler(weights, len(subset), replacement=True)
            pick = torch.multinomial(self.weights, len(idx), replacement=True, generator=self.g).tolist()
            return [idx[i] for i in pick]
        # DistributedSampler(shuffle=True): padded to a multiple of world, strided by rank
        perm = torch.randperm(len(idx), generator=self.g).tolist()
        per = -(-len(perm) // self.world)
        perm += perm[:per * self.world - len(perm)]
        return [idx[i] for i in perm[self.rank::self.world]]

    def __len__(self):
        n = len(self.subset) if self.weights is not None else -(-len(self.subset) // self.world)
        return -(-n // self.batch_size)

    def __iter__(self):
        ds = self.subset.dataset
        order = self._indices()
        for i in range(0, len(order), self.batch_size):
            yield ds.gather([ds.window_params(j) for j in order[i:i + self.batch_size]])


class DatasetLoader:
    """processing/dataset.py:264-321: split songs into train/test by
    test_ratio, weighted (length-share) sampling with replacement per rank
    (the reference's ``parallel: False`` path) or a DistributedSampler shard
    (``parallel=True``)."""

    def __init__(self, directory, metadata, batch_size=2, test_ratio=0.2, block_len=BLOCK_LEN, device="cuda",
                 parallel=False, rank=0, world=1, seed=None, **dataset_kw):
        self.directory, self.batch_size, self.test_ratio = directory, batch_size, test_ratio
        # g: split + DistributedSampler permutation, and the file shuffle
        # (identical on every rank); gs: this rank's weighted draws; the
        # dataset rng: this rank's window starts / augmentation draws
        self.g, self.gs = torch.Generator(), torch.Generator()
        if seed is not None:
            self.g.manual_seed(seed)
            self.gs.manual_seed(seed + 1000 + rank)
            dataset_kw.setdefault("shuffle_rng", random.Random(seed))
            dataset_kw.setdefault("rng", random.Random(seed + 1 + rank))
        self.dataset = SequenceDataset(directory, metadata, block_len=block_len, device=device, **dataset_kw)
        self.file_prob = self.dataset.file_prob()
        test_size = int(len(self.dataset) * test_ratio)
        self.train_dataset, self.test_dataset = random_split(self.dataset, [len(self.dataset) - test_size, test_size],
                                                             generator=self.g)
        self.parallel, self.rank, self.world = parallel, rank, world

    def _loader(self, subset):
        if self.parallel:
            return DeviceLoader(subset, self.batch_size, rank=self.rank, world=self.world, generator=self.g)
        return DeviceLoader(subset, self.batch_size, weights=[self.file_prob[i] for i in subset.indices],
                            generator=self.gs)

    def get_dataloaders(self):
        return self._loader(self.train_dataset), self._loader(self.test_dataset)

    def get_dataloader_full(self, shuffle=False):
        full = _Subset(self.dataset, range(len(self.dataset)))
        if shuffle:
            return DeviceLoader(full, self.batch_size, world=1, generator=self.g)
        return _Sequential(full, self.batch_size)


class _Sequential(DeviceLoader):
    def __init__(self, subset, batch_size):
        super().__init__(subset, batch_size)

    def _indices(self):
        return list(self.subset.indices)

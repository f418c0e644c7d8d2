"""Data feed host logic (processing/dataset.py) and its oracle, pinned to G6
(tests/golden/make_g6_data.py: the reference's own SequenceDataset run in the
build container). CPU only: metadata tokens, window draws, samplers."""
import json
import random
from pathlib import Path

import numpy as np
import pytest
import torch

from oracle import dataset as odata
from oracle.fill import REAL
from midiseq import data

G6 = np.load(Path(__file__).parent / "golden" / "g6_data.npz")
DISC = (128, 129, 128, 512, 512, 250)


def _artists():
    return json.loads(G6["artists_json"].tobytes().decode())


def test_metadata_tokens_match_reference():
    meta, tok = data.metadata_tokens({"artists": _artists()})
    names = list(G6["band_names"])
    assert list(meta) == names
    np.testing.assert_array_equal(np.array([meta[b] for b in names]), G6["band_meta"])
    ref = json.loads(G6["tokenization_json"].tobytes().decode())
    assert tok["VOCAB_SIZE"] == ref["VOCAB_SIZE"] == 568
    for key in ("time_tokenized", "genre_tokenized", "band_tokenized"):
        assert {("null" if k is None else str(k)): v for k, v in tok[key].items()} == ref[key]
    assert meta["Mozart"] == [519, 279, 202, 202, 202, 178]  # SURVEY.md §8(d) composer vectors


def _songs():
    return {k[5:].replace("__", "/"): G6[k] for k in G6.files if k.startswith("song_")}


@pytest.mark.parametrize("aug", [0, 1])
def test_oracle_samples_match_reference(aug):
    songs, T = _songs(), int(G6["T"])
    order = list(G6[f"aug{aug}_order"])
    for n, (i, ix, note, vel, f2) in enumerate(G6[f"aug{aug}_params"]):
        rep, i = divmod(n, len(order))
        src, trg = odata.sample(songs[order[i]], T, ix, (note, vel, f2 / 2) if aug else None, DISC)
        np.testing.assert_array_equal(src, G6[f"aug{aug}_src_{rep}_{i}"])
        np.testing.assert_array_equal(trg, G6[f"aug{aug}_trg_{rep}_{i}"])


def _corpus(tmp_path):
    for rel, s in _songs().items():
        p = tmp_path / rel
        p.parent.mkdir(parents=True, exist_ok=True)
        np.save(p, s)
    return tmp_path


@pytest.mark.parametrize("aug", [0, 1])
def test_window_draws_follow_reference(tmp_path, aug):
    """Same song order (os.walk + shuffle of the seeded stream) and the same
    per-sample draws (window start, then the augmentation draws)."""
    root = _corpus(tmp_path)
    ds = data.SequenceDataset(str(root), {"artists": _artists()}, block_len=int(G6["T"]), device="cpu",
                              augmentation=bool(aug), rng=random.Random(11))
    order = [str(Path(p).relative_to(root)) for p in ds.file_paths]
    if order != list(G6[f"aug{aug}_order"]):
        pytest.skip("os.walk lists this filesystem's entries in another order")
    got = [ds.window_params(i) for _ in range(4) for i in range(len(ds))]
    np.testing.assert_array_equal(np.array(got), G6[f"aug{aug}_params"])
    np.testing.assert_allclose(ds.file_prob(), ds.lengths / ds.lengths.sum())
    assert ds.song_meta.tolist()[order.index("ABBA/a.npy")] == data.metadata_tokens({"artists": _artists()})[0]["ABBA"]


def test_samplers(tmp_path):
    root = _corpus(tmp_path)
    dl = data.DatasetLoader(str(root), {"artists": _artists()}, batch_size=2, test_ratio=0.34, block_len=16,
                            device="cpu", seed=3)
    assert len(dl.train_dataset) == 2 and len(dl.test_dataset) == 1
    assert sorted(dl.train_dataset.indices + dl.test_dataset.indices) == [0, 1, 2]
    tr, te = dl.get_dataloaders()
    idx = tr._indices()
    assert len(idx) == 2 and set(idx) <= set(dl.train_dataset.indices) and len(tr) == 1
    # DistributedSampler: world shards partition one padded permutation
    shards = [data.DeviceLoader(data._Subset(None, range(7)), 2, rank=r, world=3,
                                generator=torch.Generator().manual_seed(5))._indices() for r in range(3)]
    assert all(len(s) == 3 for s in shards) and set(sum(shards, [])) == set(range(7))


@pytest.mark.parametrize("parallel", [False, True])
def test_ranks_share_split_and_shard_disjointly(tmp_path, parallel):
    """world = 2: both ranks see the same shuffled song list and train/test
    split (processing/dataset.py:66-71 shuffle, :280-288 random_split), draw
    different windows, and with parallel=True (DistributedSampler) their train
    shards partition the train songs."""
    root = tmp_path
    rng = np.random.default_rng(2)
    for b in ("ABBA", "Mozart", "Bach"):
        (root / b).mkdir()
        for k in range(4):
            np.save(root / b / f"s{k}.npy", rng.integers(0, 17914, size=int(rng.integers(40, 90))).astype(np.int64))
    arts = [a for a in _artists() if a["name"] in ("ABBA", "Mozart", "Bach")]
    dls = [data.DatasetLoader(str(root), {"artists": arts}, batch_size=2, test_ratio=0.34, block_len=16,
                              device="cpu", parallel=parallel, rank=r, world=2, seed=7) for r in range(2)]
    assert dls[0].dataset.file_paths == dls[1].dataset.file_paths
    assert dls[0].train_dataset.indices == dls[1].train_dataset.indices
    assert dls[0].test_dataset.indices == dls[1].test_dataset.indices
    draws = [[dl.dataset.window_params(i)[1] for i in range(len(dl.dataset))] for dl in dls]
    assert draws[0] != draws[1]
    if parallel:
        shards = [dl.get_dataloaders()[0]._indices() for dl in dls]
        assert not set(shards[0]) & set(shards[1])
        assert set(shards[0]) | set(shards[1]) == set(dls[0].train_dataset.indices)

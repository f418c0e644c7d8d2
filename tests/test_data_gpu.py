"""Device window gather (msq_window_gather, csrc/data.hip) against the G6
golden samples of the reference's SequenceDataset and the numpy oracle
(oracle/dataset.py): bit-exact int64 tokens, incl. zero padding of short
songs, the augmentation edge tokens and the metadata rows."""
import json
import random
from pathlib import Path

import numpy as np
import pytest
import torch

from oracle import dataset as odata
from midiseq import data

pytestmark = pytest.mark.gpu
G6 = np.load(Path(__file__).parent / "golden" / "g6_data.npz")
DISC = (128, 129, 128, 512, 512, 250)


def _artists():
    return {"artists": json.loads(G6["artists_json"].tobytes().decode())}


@pytest.mark.parametrize("aug", [0, 1])
def test_gather_matches_reference_samples(tmp_path, aug):
    songs = {k[5:].replace("__", "/"): G6[k] for k in G6.files if k.startswith("song_")}
    for rel, s in songs.items():
        p = tmp_path / rel
        p.parent.mkdir(parents=True, exist_ok=True)
        np.save(p, s)
    ds = data.SequenceDataset(str(tmp_path), _artists(), block_len=int(G6["T"]), device="cuda",
                              augmentation=bool(aug), rng=random.Random(0))
    mine = [str(Path(p).relative_to(tmp_path)) for p in ds.file_paths]
    order = list(G6[f"aug{aug}_order"])
    prm = G6[f"aug{aug}_params"].copy()
    prm[:, 0] = [mine.index(order[i]) for i in prm[:, 0]]  # golden song index -> this store's
    src, trg, meta = ds.gather(prm)
    torch.cuda.synchronize()
    for n in range(len(prm)):
        rep, i = divmod(n, len(order))
        np.testing.assert_array_equal(src[n].cpu().numpy(), G6[f"aug{aug}_src_{rep}_{i}"])
        np.testing.assert_array_equal(trg[n].cpu().numpy(), G6[f"aug{aug}_trg_{rep}_{i}"])
        np.testing.assert_array_equal(meta[n].cpu().numpy(), G6[f"aug{aug}_meta_{rep}_{i}"])


def test_gather_full_size_against_oracle(tmp_path):
    """T = 2048, 64 windows over 40 songs of 100..6000 tokens, augmentation on."""
    rng = np.random.default_rng(9)
    bands = ["ABBA", "Mozart", "Bach"]
    songs = {}
    for k in range(40):
        s = rng.integers(0, 17914, size=int(rng.integers(100, 6000))).astype(np.int64)
        rel = f"{bands[k % 3]}/s{k}.npy"
        (tmp_path / bands[k % 3]).mkdir(exist_ok=True)
        np.save(tmp_path / rel, s)
        songs[rel] = s
    ds = data.SequenceDataset(str(tmp_path), _artists(), block_len=2048, device="cuda", augmentation=True,
                              rng=random.Random(4))
    names = [str(Path(p).relative_to(tmp_path)) for p in ds.file_paths]
    prm = [ds.window_params(int(i)) for i in rng.integers(0, len(ds), size=64)]
    src, trg, meta = ds.gather(prm)
    torch.cuda.synchronize()
    mt = data.metadata_tokens(_artists())[0]
    for b, (i, ix, note, vel, f2) in enumerate(prm):
        rs, rt = odata.sample(songs[names[i]], 2048, ix, (note, vel, f2 / 2), DISC)
        np.testing.assert_array_equal(src[b].cpu().numpy(), rs)
        np.testing.assert_array_equal(trg[b].cpu().numpy(), rt)
        assert meta[b].tolist() == mt[names[i].split("/")[0]]


def test_loader_batches_feed_the_train_step(tmp_path):
    rng = np.random.default_rng(1)
    for k in range(6):
        (tmp_path / "Mozart").mkdir(exist_ok=True)
        np.save(tmp_path / "Mozart" / f"m{k}.npy", rng.integers(0, 17914, size=3000).astype(np.int64))
    dl = data.DatasetLoader(str(tmp_path), _artists(), batch_size=4, test_ratio=0.2, block_len=256,
                            device="cuda", seed=0)
    train, test = dl.get_dataloaders()
    src, trg, meta = next(iter(train))
    assert src.shape == (4, 256) and trg.shape == (4, 256) and meta.shape == (4, 6)
    assert src.dtype == torch.int64 and src.is_cuda
    assert torch.equal(src[:, 1:], trg[:, :-1])
    assert (meta == torch.tensor([519, 279, 202, 202, 202, 178], device="cuda")).all()

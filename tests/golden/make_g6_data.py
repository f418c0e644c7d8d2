"""G6 golden vectors for the data feed, from the REFERENCE's own
processing/dataset.py (build container only; the reference never travels).

Run:  python tests/golden/make_g6_data.py [/root/reference]

Records into tests/golden/g6_data.npz:
  * the metadata vectors of every band and the tokenization tables that
    SequenceDataset.get_metadata_dict (dataset.py:76-132) derives from the
    reference's metadata.json (input artists kept as data);
  * __getitem__ samples (dataset.py:171-195) of a synthetic 3-song corpus
    (shorter than, equal to and longer than the window), with and without
    data_augementation (:134-168), each with the random draws that produced it.
"""
import json
import random
import sys
import tempfile
import types
from pathlib import Path

import numpy as np
import torch

REPO = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(REPO / "tests" / "golden"))
sys.path.insert(0, str(REPO))
from make_golden import RefShim, ns  # noqa: E402
from oracle.fill import Vocab  # noqa: E402

OUT = REPO / "tests" / "golden" / "g6_data.npz"


def main(ref=Path(sys.argv[1] if len(sys.argv) > 1 else "/root/reference")):
    vocab = Vocab()
    sh = RefShim(ref, vocab, 568)
    tmp = Path(tempfile.mkdtemp())
    paths = sys.modules["configs.paths"]
    paths.config = ns({"paths": {"metadata": str(ref / "metadata.json"), "tokenizations": str(tmp / "tok.json"),
                                 "pretrained": "/nonexistent"}})
    sys.modules["configs"].paths = paths
    ds_mod = sh._load("ref_dataset", "processing/dataset.py")
    meta = ds_mod.SequenceDataset.get_metadata_dict(None)
    tok = json.load(open(tmp / "tok.json"))
    artists = json.load(open(ref / "metadata.json"))["artists"]
    out = {
        "artists_json": np.frombuffer(json.dumps(artists).encode(), dtype=np.uint8),
        "band_names": np.array(list(meta.keys())),
        "band_meta": np.stack([meta[b].numpy() for b in meta]).astype(np.int64),
        "tokenization_json": np.frombuffer(json.dumps(tok).encode(), dtype=np.uint8),
    }
    # synthetic corpus: band dirs from metadata.json, songs of 10 / 17 / 40 tokens
    T = 16
    sh.cc.config.values.block_len = T
    rng = np.random.default_rng(6)
    lens = {"ABBA/a.npy": 10, "ABBA/b.npy": T + 1, "2_Unlimited/c.npy": 40}
    corpus = tmp / "corpus"
    songs = {}
    for rel, n in lens.items():
        p = corpus / rel
        p.parent.mkdir(parents=True, exist_ok=True)
        s = rng.integers(0, vocab.size, size=n).astype(np.int64)
        # make every augmentation range and its edges appear
        st = vocab.start
        edges = [0, 127, 128, 16510, 16511, st["dyn"], st["dyn"] + 126, st["dyn"] + 127, st["length"],
                 st["length"] + 510, st["length"] + 511, st["time"], st["time"] + 510, st["time"] + 511,
                 st["tempo"], st["tempo"] + 248, st["tempo"] + 249]
        s[:min(n, len(edges))] = edges[:min(n, len(edges))]
        np.save(p, s)
        songs[rel] = s
    for aug in (False, True):
        sh.cc.config.values.augmentation = aug
        random.seed(11)
        ds = ds_mod.SequenceDataset(str(corpus))
        order = [str(Path(p).relative_to(corpus)) for p in ds.file_paths]
        samples = []
        for rep in range(4):
            for i in range(len(ds)):
                st_ = random.getstate()
                n = len(songs[order[i]])
                ix = random.randint(0, n - (T + 1)) if n > T + 1 else 0
                draws = (random.randint(-12, 12), random.randint(-20, 20), random.randint(1, 8)) if aug else (0, 0, 2)
                random.setstate(st_)
                src, trg, m = ds[i]
                samples.append((i, ix) + draws)
                out[f"aug{int(aug)}_src_{rep}_{i}"] = src.numpy()
                out[f"aug{int(aug)}_trg_{rep}_{i}"] = trg.numpy()
                out[f"aug{int(aug)}_meta_{rep}_{i}"] = m.numpy()
        out[f"aug{int(aug)}_order"] = np.array(order)
        out[f"aug{int(aug)}_params"] = np.array(samples, dtype=np.int64)
    for rel, s in songs.items():
        out["song_" + rel.replace("/", "__")] = s
    out["T"] = np.array(T)
    np.savez_compressed(OUT, **out)
    print("wrote", OUT, len(out), "arrays")


if __name__ == "__main__":
    main()

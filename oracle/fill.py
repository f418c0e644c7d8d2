"""Deterministic, platform-independent weight and input generators (test infra).

Weights are produced from a splitmix64 integer hash of (element index, salt), so
the golden-vector generator (which runs the reference) and the parity tests
(which run the HIP path) build bit-identical parameters without sharing any
torch RNG state. Token inputs follow the MIDI grammar of SURVEY.md §8(d).
"""
import zlib

import numpy as np

_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)
_G = np.uint64(0x9E3779B97F4A7C15)


def hash_uniform(n: int, salt: int) -> np.ndarray:
    """n values uniform in [-0.5, 0.5), exactly representable in fp32."""
    with np.errstate(over="ignore"):
        z = np.arange(n, dtype=np.uint64) + np.uint64(salt & 0xFFFFFFFF) * _G
        z = (z ^ (z >> np.uint64(30))) * _M1
        z = (z ^ (z >> np.uint64(27))) * _M2
        z = z ^ (z >> np.uint64(31))
    return ((z >> np.uint64(40)).astype(np.float64) / float(1 << 24)) - 0.5


def name_salt(name: str) -> int:
    return zlib.crc32(name.encode())


def fill_param(name: str, shape) -> np.ndarray:
    """fp32 array for a reference state_dict key (names of model_transformer.py
    / mamba.py). Scales roughly follow the modules' default inits."""
    n = int(np.prod(shape))
    u = hash_uniform(n, name_salt(name)).reshape(shape)
    leaf = name.rsplit(".", 1)[-1]
    if "embedding" in name or leaf == "rel_pos_emb":
        a = 2.0 * u
    elif ("ln" in name.split(".")[-2] if "." in name else False) or name.startswith("norm.") or ".norm." in name:
        a = (1.0 + 0.2 * u) if leaf == "weight" else 0.2 * u
    elif leaf == "A_log":
        a = np.log(1.0 + 15.0 * (u + 0.5))
    elif leaf == "dt_bias":
        a = -3.0 + 2.0 * u
    elif leaf == "D":
        a = 1.0 + 0.2 * u
    elif leaf == "bias":
        a = 0.1 * u
    elif leaf == "weight" and len(shape) == 3:  # depthwise conv1d [C,1,k]
        a = 2.0 * u / np.sqrt(shape[-1])
    elif leaf == "weight" and len(shape) == 2:
        a = 2.0 * u / np.sqrt(shape[1])
    else:
        a = u
    return a.astype(np.float32)


class Vocab:
    """Token-class layout of configs/common/__init__.py:31-57."""

    def __init__(self, pitch=128, channel=129, dyn=128, length=512, time=512, tempo=250):
        self.disc = dict(pitch=pitch, channel=channel, dyn=dyn, length=length, time=time, tempo=tempo)
        self.start = {}
        off = 0
        for key, width in (("pitch", pitch * channel), ("dyn", dyn), ("length", length),
                           ("time", time), ("tempo", tempo)):
            self.start[key] = off
            off += width
        self.size = off


REAL = Vocab()
TINY = Vocab(pitch=4, channel=2, dyn=4, length=8, time=8, tempo=6)


def grammar_tokens(rng: np.random.Generator, vocab: Vocab, n: int) -> np.ndarray:
    """Grammar-cycled synthetic MIDI tokens: pitch, dyn, length,
    optional time (p=0.5), tempo. Includes the per-class last tokens sometimes."""
    s = vocab.start
    out = []
    while len(out) < n:
        out.append(int(rng.integers(s["pitch"], s["dyn"])))
        out.append(int(rng.integers(s["dyn"], s["length"])))
        out.append(int(rng.integers(s["length"], s["time"])))
        if rng.random() < 0.5:
            out.append(int(rng.integers(s["time"], s["tempo"])))
        out.append(int(rng.integers(s["tempo"], vocab.size)))
    return np.asarray(out[:n], dtype=np.int64)


COMPOSERS = {
    # meta vectors derived from metadata.json + tokenization.json
    "mozart": [519, 279, 202, 202, 202, 178],
    "bach": [432, 277, 202, 202, 202, 173],
    "beethoven": [437, 279, 272, 202, 202, 180],
    "chopin": [452, 272, 202, 202, 202, 184],
    "liszt": [508, 272, 202, 202, 202, 184],
}

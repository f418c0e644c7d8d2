"""Vocabulary layout and default hyper-parameters (configs/common/__init__.py:
31-57, configs/common/config.yaml, configs/transformer/config.yaml).

The reference computes these at import time from YAML plus a hard-coded
/scratch tokenization file; here they are plain values, overridable per
instance (the parity tests use a tiny vocabulary)."""
from dataclasses import dataclass, field

import torch


@dataclass
class Discretization:
    pitch: int = 128
    channel: int = 129  # 128 instruments + drums
    dyn: int = 128
    length: int = 512
    time: int = 512
    tempo: int = 250

    @property
    def vocab_size(self) -> int:
        return self.pitch * self.channel + self.dyn + self.length + self.time + self.tempo

    @property
    def start_idx(self) -> dict:
        off, out = 0, {}
        for k, w in (("pitch", self.pitch * self.channel), ("dyn", self.dyn), ("length", self.length),
                     ("time", self.time), ("tempo", self.tempo)):
            out[k] = off
            off += w
        return out


DEFAULT_DISC = Discretization()
VOCAB_SIZE = DEFAULT_DISC.vocab_size          # 17 914
METADATA_VOCAB_SIZE = 568                     # tokenization.json VOCAB_SIZE
BLOCK_LEN = 2048                              # config.yaml values.block_len
N_META = 6                                    # metadata tokens per piece
LEARNING_RATE = 5e-5                          # config.yaml values.learning_rate
DROPOUT = 0.01                                # config.yaml values.dropout
EPOCHS = 10000                                # config.yaml values.epochs
EVAL_INTERVAL = 10                            # config.yaml values.eval_interval (steps between loss logs)
SAVE_INTERVAL = 10                            # config.yaml values.save_interval (epochs between saves)
TEST_RATIO = 0.2                              # config.yaml values.test_ratio
BATCH_SIZE = 2                                # config.yaml values.batch_size


@dataclass
class Grammar:
    """The 5 x V weight table of make_distributions (train.py:79-111) and the
    bucketize boundaries of pick_distributions_by_prev_token (:114-131)."""
    disc: Discretization = field(default_factory=Discretization)

    @property
    def bounds(self):
        s = self.disc.start_idx
        return (s["dyn"] - 1, s["length"] - 1, s["time"] - 1, s["tempo"] - 1)

    def table(self, device="cpu") -> torch.Tensor:
        s, V = self.disc.start_idx, self.disc.vocab_size
        t = torch.zeros(5, V, dtype=torch.float32)
        t[0, s["dyn"]:s["length"] - 1] = 1.0                                   # after pitch: dynamics
        t[1, s["length"]:s["time"] - 1] = torch.linspace(1, 3, self.disc.length - 1)  # after dyn: lengths
        t[2, s["time"]:s["tempo"] - 1] = 1.0                                   # after length: time ...
        t[2, s["tempo"]:V] = 1.0                                               # ... or tempo
        t[3, s["tempo"]:V] = 1.0                                               # after time: tempo
        t[4, s["pitch"]:s["dyn"] - 1] = 10.0                                   # after tempo: pitch x10
        return t.to(device)

"""CPU oracle (test infra) for the grammar-weighted "filtered" loss.

Restates train.py:79-138 (== train_parallel.py:83-141) and the
CrossEntropyLoss call of train_parallel.py:156,179.
"""
import numpy as np
import torch

from .fill import Vocab


def weight_table(v: Vocab) -> np.ndarray:
    """5 x V table of train.py:79-111.

    Row r is selected by the class of the *previous* token (bucket r). The
    reference slices ``start:end`` with ``end = next_start - 1``, so the last
    token of every class except tempo is excluded (train.py:91-95).
    """
    s = v.start
    V = v.size
    tab = np.zeros((5, V), dtype=np.float32)
    tab[0, s["dyn"]:s["length"] - 1] = 1.0            # after pitch  -> dynamics
    tab[1, s["length"]:s["time"] - 1] = torch.linspace(  # after dyn -> lengths (train.py:18,107)
        1, 3, steps=v.disc["length"] - 1).numpy()
    tab[2, s["time"]:s["tempo"] - 1] = 1.0            # after length -> time
    tab[2, s["tempo"]:V] = 1.0                        #              or tempo (train.py:99)
    tab[3, s["tempo"]:V] = 1.0                        # after time   -> tempo
    tab[4, s["pitch"]:s["dyn"] - 1] = 10.0            # after tempo  -> pitch x10 (train.py:109)
    return tab


def weight_table_torch(v: Vocab) -> torch.Tensor:
    return torch.from_numpy(weight_table(v))


def bucket_of(tokens: np.ndarray, v: Vocab) -> np.ndarray:
    """torch.bucketize(x, [dyn-1, length-1, time-1, tempo-1], right=False)
    (train.py:117-124): number of boundaries strictly below x."""
    s = v.start
    bounds = np.array([s["dyn"] - 1, s["length"] - 1, s["time"] - 1, s["tempo"] - 1], dtype=np.int64)
    return (tokens[..., None] > bounds).sum(-1).astype(np.int64)


def filtered_logit(src: torch.Tensor, logits: torch.Tensor, v: Vocab) -> torch.Tensor:
    """Z = -(o - LSE_t o) * W[bucket(src)] — log-softmax over the TIME axis
    (dim=1), train.py:133-138."""
    w = weight_table_torch(v)[torch.from_numpy(bucket_of(src.numpy(), v))]
    lse_t = torch.logsumexp(logits, dim=1, keepdim=True)
    return -(logits - lse_t) * w


def loss(src, trg, logits, v: Vocab) -> torch.Tensor:
    """mean over B*T of LSE_v(Z) - Z[y]; no ignore_index (train_parallel.py:156,179)."""
    z = filtered_logit(src, logits, v).reshape(-1, v.size)
    y = trg.reshape(-1)
    return (torch.logsumexp(z, dim=-1) - z.gather(1, y[:, None])[:, 0]).mean()

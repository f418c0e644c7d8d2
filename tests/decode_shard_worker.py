"""Worker of tests/test_decode_shard_gpu.py (not a test module): one rank of
a world-2 sharded decode (generate(..., group=True)) on the ONE leased GPU,
process group gloo. Rank r decodes rows r*B .. r*B+B-1 of the global prompt
batch and writes them to <out>_<r>.npz.

usage (under torch.distributed.run): decode_shard_worker.py <exact|cached> <out prefix>"""
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import _pkgload  # noqa: E402

_pkgload.load()
from midiseq.generate import generate  # noqa: E402
from midiseq.train_parallel import setup_distributed  # noqa: E402

HP = dict(n_embd=64, n_heads=4, n_layer=2, block_len=48)
STEPS, B_GLOBAL, T0 = 8, 4, 40


def build_model():
    from oracle import transformer as otr
    from oracle.fill import REAL
    from midiseq.transformer import Transformer, TransformerConfig
    m = Transformer(TransformerConfig(vocab_size=REAL.size, metadata_vocab_size=568, precision="fp32", dropout=0.0,
                                      **HP)).to("cuda").eval()
    m.load_state_dict(otr.filled_params(otr.param_shapes(HP["n_embd"], HP["n_heads"], HP["n_layer"],
                                                         HP["block_len"], REAL.size, 568)))
    return m


def prompts():
    from oracle.fill import REAL, grammar_tokens
    rng = np.random.default_rng(17)
    src = np.stack([grammar_tokens(rng, REAL, T0) for _ in range(B_GLOBAL)])
    meta = np.array([[519, 279, 202, 202, 202, 178], [432, 277, 202, 202, 202, 173],
                     [437, 279, 272, 202, 202, 180], [452, 272, 202, 202, 202, 184]])
    us = rng.random(B_GLOBAL * STEPS).tolist()
    return torch.from_numpy(src), torch.from_numpy(meta), us


def run(model, src, meta, mode, uniforms, group=None):
    """(rows with recorded uniforms, rows from torch's seeded generator)"""
    a = generate(model, HP["block_len"], src, meta, num_tokens=STEPS, rng=random.Random(5), uniforms=iter(uniforms),
                 mode=mode, group=group)
    torch.manual_seed(123)
    b = generate(model, HP["block_len"], src, meta, num_tokens=STEPS, rng=random.Random(6), mode=mode, group=group)
    return np.array(a), np.array(b)


def main():
    mode, out = sys.argv[1], sys.argv[2]
    rank, _, world = setup_distributed(backend="gloo")
    assert world == 2
    torch.cuda.set_device(0)
    model = build_model()
    src, meta, us = prompts()
    n = B_GLOBAL // world
    a, b = run(model, src[rank * n:(rank + 1) * n], meta[rank * n:(rank + 1) * n], mode, us, group=True)
    np.savez(f"{out}_{rank}.npz", a=a, b=b)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()

"""Times the secondary paths: Mamba train step (cfg 3: d=1024, 10 layers,
T=4096, B=8) and exact sliding-window decode (cfg 5: B=64 prompts of 2048).
Usage: python tools/bench_paths.py [mamba|decode|all] [steps]"""
import os
import random
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import _pkgload  # noqa: E402

_pkgload.load()
import torch  # noqa: E402

from midiseq.train_parallel import TrainStep, SyntheticMIDI  # noqa: E402


def mamba(steps=3, B=8, T=4096):
    from midiseq.mamba import Mamba
    m = Mamba(precision="bf16").to("cuda")
    st = TrainStep(m)
    data = iter(SyntheticMIDI(B, T, torch.device("cuda"), 0, n_batches=2))
    st(*next(data))
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        loss = st(*next(data))
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    print(f"mamba train B={B} T={T}: {dt*1e3:.1f} ms/step, {B*T/dt:.0f} tok/s, loss {loss.item():.3f}")


def decode(steps=4, B=64, T=2048):
    from midiseq.transformer import Transformer, TransformerConfig
    from midiseq.generate import generate
    m = Transformer(TransformerConfig(precision="bf16")).to("cuda")
    data = SyntheticMIDI(B, T, torch.device("cuda"), 0, n_batches=1)
    src, _, meta = data.batches[0]
    generate(m, T, src, meta, num_tokens=1, rng=random.Random(0))
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    generate(m, T, src, meta, num_tokens=steps, rng=random.Random(0))
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    print(f"decode B={B} ctx={T}: {dt*1e3:.1f} ms/step, {B/dt:.1f} new tok/s")


if __name__ == "__main__":
    which = sys.argv[1] if len(sys.argv) > 1 else "all"
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    if which in ("mamba", "all"):
        mamba(n)
    if which in ("decode", "all"):
        decode(n)

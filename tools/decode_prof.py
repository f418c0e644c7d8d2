"""Decode-step timing (GPU only): the Mamba recurrent step and the Transformer
cached step at B=64, replayed as HIP graphs vs launched eagerly, beside the
whole generate() iteration (sampling, host k choice, one D2H sync).

  python tools/decode_prof.py [mamba|transformer] [steps]"""
import os
import random
import sys
import time
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import _pkgload  # noqa: E402

_pkgload.load()
from midiseq.generate import generate  # noqa: E402
from midiseq.train_parallel import SyntheticMIDI  # noqa: E402


def ev_time(fn, n):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n


def main(kind="mamba", n=50):
    dev = "cuda"
    B, T0 = 64, int(os.environ.get("DP_T0", 1024))
    if kind == "mamba":
        from midiseq.mamba import Mamba
        m = Mamba(precision="bf16").to(dev)
    else:
        from midiseq.transformer import Transformer, TransformerConfig
        m = Transformer(TransformerConfig(precision="bf16", dropout=0.0)).to(dev).eval()
    eng = m.engine
    src, _, meta = SyntheticMIDI(B, T0, dev, 0, n_batches=1).batches[0]
    tok = src[:, -1].contiguous()
    with torch.no_grad():
        cache = eng.decode_cache(B, 2048) if kind != "mamba" else eng.decode_cache(B)
        eng.forward(src, meta, save=False, cache=cache)
        if kind == "mamba":
            eng.step_graphs = False
            eager = ev_time(lambda: eng.step(tok, cache), n)
            eng.step_graphs = True
            graph = ev_time(lambda: eng.step(tok, cache), n)
            print(f"mamba step: eager {eager:.3f} ms, graph {graph:.3f} ms", flush=True)
        else:
            eager = ev_time(lambda: eng.step(tok, cache), n)
            print(f"transformer cached step: eager {eager:.3f} ms", flush=True)
    K = 32
    run = lambda k: generate(m, 2048, src, meta, num_tokens=k, rng=random.Random(0), device=dev,  # noqa: E731
                             mode="cached", return_tensor=True)
    run(2)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run(1)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    run(1 + K)
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"generate iteration: {((t2 - t1) - (t1 - t0)) / K * 1e3:.3f} ms per new token (B={B})", flush=True)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "mamba", int(sys.argv[2]) if len(sys.argv) > 2 else 50)

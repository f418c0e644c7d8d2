"""Generate golden vectors from the REFERENCE's own code (build container only).

Run:  python tests/golden/make_golden.py [/root/reference]

The reference cannot be imported as-is (hard-coded /scratch paths, device
'cuda', an import-time ``.to("cuda")`` in train.py, and mamba_ssm/pretty_midi
imports). This script builds a throw-away ``configs.common`` module from the
reference's own config.yaml + tokenization.json (device forced to cpu, dropout
forced to 0), loads model_transformer.py, train.py and scripts/generate.py by
file path with the unrelated imports stubbed, and records their outputs on
deterministic inputs into tests/golden/*.npz. Only data is written; nothing
from the reference is copied into the repository.
"""
import importlib.machinery
import importlib.util
import json
import os
import random
import sys
import types
from pathlib import Path

import numpy as np
import torch
import yaml

REPO = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(REPO))
from oracle.fill import Vocab, fill_param, grammar_tokens, COMPOSERS  # noqa: E402
from oracle import transformer as otr  # noqa: E402

OUT = REPO / "tests" / "golden"


def ns(d):
    if isinstance(d, dict):
        return types.SimpleNamespace(**{k: ns(v) for k, v in d.items()})
    return d


class RefShim:
    """Loads reference modules by path against a synthetic configs.common."""

    def __init__(self, ref: Path, vocab: Vocab, meta_vocab: int):
        self.ref = ref
        cfg = yaml.safe_load(open(ref / "configs/common/config.yaml"))
        cfg["values"]["device"] = "cpu"
        cfg["values"]["dropout"] = 0.0
        for k, val in vocab.disc.items():
            cfg["discretization"][k] = val
        toks = json.load(open(ref / "tokenization.json"))
        cc = types.ModuleType("configs.common")
        cc.config = ns(cfg)
        cc.tokenizations = ns(toks)
        cc.vocab_size = vocab.size
        cc.metadata_vocab_size = meta_vocab
        cc.start_idx = dict(vocab.start)
        configs = types.ModuleType("configs")
        configs.__path__ = []
        configs.common = cc
        for name in ("mamba", "xlstm", "transformer", "paths"):
            m = types.ModuleType("configs." + name)
            m.config = ns({"model_values": {}, "paths": {"pretrained": "/nonexistent"}})
            setattr(configs, name, m)
            sys.modules["configs." + name] = m
        sys.modules["configs"] = configs
        sys.modules["configs.common"] = cc
        for stub in ("models", "processing", "mamba_ssm", "pretty_midi"):
            if stub == "mamba_ssm" and hasattr(sys.modules.get(stub), "Mamba2"):
                continue
            sys.modules[stub] = types.ModuleType(stub)
            sys.modules[stub].__spec__ = importlib.machinery.ModuleSpec(stub, None)
        self.cc = cc
        self.mt = self._load("ref_model_transformer", "models/transformer/model_transformer.py")
        orig_to = torch.Tensor.to

        def to_cpu(t, *a, **k):  # train.py:18 calls .to("cuda") at import
            a = tuple("cpu" if x == "cuda" else x for x in a)
            return orig_to(t, *a, **k)
        torch.Tensor.to = to_cpu
        try:
            self.train = self._load("train", "train.py")
        finally:
            torch.Tensor.to = orig_to
        sys.modules["train"] = self.train
        self.gen = self._load("ref_generate", "scripts/generate.py")

    def _load(self, name, rel):
        spec = importlib.util.spec_from_file_location(name, self.ref / rel)
        mod = importlib.util.module_from_spec(spec)
        sys.modules[name] = mod
        spec.loader.exec_module(mod)
        return mod

    def transformer(self, n_embd, n_heads, n_layer, block_len):
        p = types.SimpleNamespace(n_embd=n_embd, n_heads=n_heads, n_layer=n_layer, block_len=block_len,
                                  dropout=0.0, vocab_size=self.cc.vocab_size,
                                  metadata_vocab_size=self.cc.metadata_vocab_size, device="cpu")
        m = self.mt.Transformer(p)
        shapes = otr.param_shapes(n_embd, n_heads, n_layer, block_len, self.cc.vocab_size,
                                  self.cc.metadata_vocab_size)
        sd = m.state_dict()
        for k, s in shapes.items():
            assert tuple(sd[k].shape) == tuple(s), (k, sd[k].shape, s)
            sd[k] = torch.from_numpy(fill_param(k, s))
        m.load_state_dict(sd)
        assert set(shapes) | {k for k in sd if k.endswith("tril")} == set(sd), "state_dict key mismatch"
        return m


def projection(V, k=8, salt=7):
    from oracle.fill import hash_uniform
    return torch.from_numpy(hash_uniform(V * k, salt).reshape(V, k).astype(np.float32))


def make_inputs(vocab, B, T, meta_vocab, seed):
    rng = np.random.default_rng(seed)
    w = np.stack([grammar_tokens(rng, vocab, T + 1) for _ in range(B)])
    if meta_vocab >= 568:
        names = list(COMPOSERS)
        meta = np.array([COMPOSERS[names[b % len(names)]] for b in range(B)], dtype=np.int64)
    else:
        meta = rng.integers(0, meta_vocab, size=(B, 6)).astype(np.int64)
    return w[:, :-1].copy(), w[:, 1:].copy(), meta


def g1_g2(ref_path):
    out = {}
    for tag, vocab in (("tiny", Vocab(pitch=4, channel=2, dyn=4, length=8, time=8, tempo=6)), ("real", Vocab())):
        sh = RefShim(ref_path, vocab, 568)
        tab = sh.train.make_distributions().numpy()
        out[f"{tag}_table_nz_idx"] = np.nonzero(tab.reshape(-1))[0].astype(np.int64)
        out[f"{tag}_table_nz_val"] = tab.reshape(-1)[np.nonzero(tab.reshape(-1))[0]]
        s = vocab.start
        edges = []
        for key in ("pitch", "dyn", "length", "time", "tempo"):
            st = s[key]
            edges += [st, st + 1]
        edges += [s["dyn"] - 1, s["length"] - 1, s["time"] - 1, s["tempo"] - 1, vocab.size - 1]
        edges = np.array(sorted(set(edges)), dtype=np.int64)
        bins = torch.tensor([s["dyn"] - 1, s["length"] - 1, s["time"] - 1, s["tempo"] - 1])
        out[f"{tag}_edge_tokens"] = edges
        out[f"{tag}_edge_buckets"] = torch.bucketize(torch.from_numpy(edges), bins, right=False).numpy()
        # filtered_logit + CE on hashed logits
        B, T = 2, 16
        from oracle.fill import hash_uniform
        logits = torch.from_numpy((4.0 * hash_uniform(B * T * vocab.size, 99)).astype(np.float32)).reshape(
            B, T, vocab.size).requires_grad_(True)
        src, trg, _ = make_inputs(vocab, B, T, 568, 5)
        src_t, trg_t = torch.from_numpy(src), torch.from_numpy(trg)
        z = sh.train.filtered_logit(src_t, logits)
        loss = torch.nn.CrossEntropyLoss()(z.reshape(-1, vocab.size), trg_t.view(-1))
        loss.backward()
        out[f"{tag}_ce_src"], out[f"{tag}_ce_trg"] = src, trg
        out[f"{tag}_ce_loss"] = np.array(loss.item(), dtype=np.float64)
        if tag == "tiny":
            out[f"{tag}_ce_z"] = z.detach().numpy()
            out[f"{tag}_ce_dlogits"] = logits.grad.numpy()
        else:
            P = projection(vocab.size)
            out[f"{tag}_ce_z_proj"] = (z.detach() @ P).numpy()
            out[f"{tag}_ce_dlogits_proj"] = (logits.grad @ P).numpy()
            out[f"{tag}_ce_z_rows"] = z.detach()[:, [0, T - 1], :].numpy()
            out[f"{tag}_ce_dlogits_rows"] = logits.grad[:, [0, 7, T - 1], :].numpy()
    np.savez_compressed(OUT / "g1g2_loss.npz", **out)


def g3(ref_path):
    out = {}
    cases = {
        "tiny": (Vocab(pitch=4, channel=2, dyn=4, length=8, time=8, tempo=6), 10, dict(n_embd=32, n_heads=4, n_layer=2, block_len=16), 2, 16),
        "small": (Vocab(), 568, dict(n_embd=128, n_heads=8, n_layer=2, block_len=64), 2, 64),
    }
    for tag, (vocab, mv, hp, B, T) in cases.items():
        sh = RefShim(ref_path, vocab, mv)
        m = sh.transformer(**hp)
        m.train()
        src, trg, meta = make_inputs(vocab, B, T, mv, 11)
        logits = m(torch.from_numpy(src), torch.from_numpy(meta))
        z = sh.train.filtered_logit(torch.from_numpy(src), logits)
        loss = torch.nn.CrossEntropyLoss()(z.reshape(-1, vocab.size), torch.from_numpy(trg).view(-1))
        m.zero_grad()
        loss.backward()
        out[f"{tag}_src"], out[f"{tag}_trg"], out[f"{tag}_meta"] = src, trg, meta
        out[f"{tag}_loss"] = np.array(loss.item(), dtype=np.float64)
        grads = {k: p.grad for k, p in m.named_parameters()}
        if tag == "tiny":
            out[f"{tag}_logits"] = logits.detach().numpy()
            for k, g in grads.items():
                out[f"{tag}_grad:{k}"] = g.numpy()
        else:
            P = projection(vocab.size)
            out[f"{tag}_logits_proj"] = (logits.detach() @ P).numpy()
            out[f"{tag}_logits_rows"] = logits.detach()[:, [0, T // 2, T - 1], :].numpy()
            for k, g in grads.items():
                gf = g.reshape(-1).double()
                out[f"{tag}_gsum:{k}"] = np.array([gf.sum().item(), gf.abs().sum().item(), (gf * gf).sum().item()])
                out[f"{tag}_gpick:{k}"] = g.reshape(-1)[:: max(1, gf.numel() // 64)][:64].numpy()
        # G6 length anchoring: drop the last token; the shared prefix's logits change
        with torch.no_grad():
            l2 = m(torch.from_numpy(src[:, :-1].copy()), torch.from_numpy(meta))
        out[f"{tag}_anchor_short_logits_row0"] = l2[:, 0].numpy()
        out[f"{tag}_anchor_maxdiff"] = np.array((l2 - logits.detach()[:, :T - 1]).abs().max().item())
    np.savez_compressed(OUT / "g3_transformer.npz", **out)


def g4(ref_path):
    out = {}
    cases = {
        "tiny": (Vocab(pitch=4, channel=2, dyn=4, length=8, time=8, tempo=6), 10, dict(n_embd=32, n_heads=4, n_layer=2, block_len=16), 3, 16, 12),
        "small": (Vocab(), 568, dict(n_embd=64, n_heads=4, n_layer=2, block_len=48), 3, 48, 8),
    }
    for tag, (vocab, mv, hp, B, T, steps) in cases.items():
        sh = RefShim(ref_path, vocab, mv)
        m = sh.transformer(**hp)
        src, _, meta = make_inputs(vocab, B, T, mv, 21)
        urng = np.random.default_rng(77)
        uniforms = urng.random(B * steps)
        it = iter(uniforms.tolist())
        trace = []
        orig_mult, orig_topk = torch.multinomial, torch.topk

        def inv_cdf(probs, n):
            u = next(it)
            c = torch.cumsum(probs, 0)
            hit = (c > u).nonzero()
            return torch.tensor([int(hit[0, 0]) if hit.numel() else probs.numel() - 1])

        def rec_topk(x, k, *a, **kw):
            r = orig_topk(x, k, *a, **kw)
            trace.append((int(k), r[1].tolist(), r[0].tolist()))
            return r
        torch.multinomial, torch.topk = inv_cdf, rec_topk
        random.seed(1234)
        try:
            seqs = sh.gen.generate(m, hp["block_len"], torch.from_numpy(src), torch.from_numpy(meta),
                                   num_tokens=steps, device="cpu")
        finally:
            torch.multinomial, torch.topk = orig_mult, orig_topk
        out[f"{tag}_src"], out[f"{tag}_meta"] = src, meta
        out[f"{tag}_uniforms"] = uniforms
        out[f"{tag}_seqs"] = np.array(seqs, dtype=np.int64)
        out[f"{tag}_k"] = np.array([t[0] for t in trace], dtype=np.int64)
        kk = np.zeros((len(trace), 3), dtype=np.int64) - 1
        pp = np.zeros((len(trace), 3), dtype=np.float32)
        for n, (k, idx, vals) in enumerate(trace):
            kk[n, :k] = idx
            pp[n, :k] = vals
        out[f"{tag}_topk_idx"], out[f"{tag}_topk_vals"] = kk, pp
    np.savez_compressed(OUT / "g4_generate.npz", **out)


def _hf_mamba2_stub():
    """mamba_ssm.Mamba2 stand-in: HF transformers' pure-torch Mamba2Mixer with
    mamba_ssm's defaults (headdim 64, ngroups 1, chunk 256, no bias, conv
    bias, rmsnorm eps 1e-5, norm_before_gate=False, dt_limit (0, inf))."""
    from transformers.models.mamba2.configuration_mamba2 import Mamba2Config
    from transformers.models.mamba2.modeling_mamba2 import Mamba2Mixer

    class Mamba2(Mamba2Mixer):
        def __init__(self, d_model, d_state=64, d_conv=4, expand=2, layer_idx=0, headdim=64, ngroups=1, **kw):
            cfg = Mamba2Config(hidden_size=d_model, state_size=d_state, conv_kernel=d_conv, expand=expand,
                               head_dim=headdim, num_heads=expand * d_model // headdim, n_groups=ngroups,
                               use_bias=False, use_conv_bias=True, chunk_size=256, layer_norm_epsilon=1e-5,
                               time_step_limit=(0.0, float("inf")), num_hidden_layers=max(1, layer_idx + 1))
            super().__init__(cfg, layer_idx)

        def forward(self, x):
            return super().forward(x)

    m = types.ModuleType("mamba_ssm")
    m.Mamba2 = Mamba2
    for name in ("mamba_ssm.utils", "mamba_ssm.utils.generation"):
        sys.modules[name] = types.ModuleType(name)
    sys.modules["mamba_ssm.utils.generation"].InferenceParams = object
    sys.modules["mamba_ssm"] = m


def g5(ref_path):
    """Reference Mamba (models/mamba/mamba.py) fwd/bwd with HF-backed Mamba2."""
    from oracle import mamba2 as om
    os.environ.setdefault("HF_HUB_OFFLINE", "1")
    out = {}
    vocab = Vocab()
    sh = RefShim(ref_path, vocab, 568)
    _hf_mamba2_stub()
    orig_to = torch.nn.Module.to

    def to_cpu(mod, *a, **k):
        a = tuple("cpu" if x == "cuda" else x for x in a)
        return orig_to(mod, *a, **k)
    torch.nn.Module.to = to_cpu
    try:
        mm = sh._load("ref_mamba", "models/mamba/mamba.py")
        full = mm.Mamba()  # defaults d_model=1024, n_layers=10
        out["default_param_count"] = np.array(sum(p.numel() for p in full.parameters()), dtype=np.int64)
        del full
        d_model, n_layers, T, B = 128, 2, 300, 2
        m = mm.Mamba(d_model=d_model, n_layers=n_layers)
    finally:
        torch.nn.Module.to = orig_to
    shapes = om.param_shapes(d_model, n_layers, vocab.size, 568)
    sd = m.state_dict()
    assert set(sd) == set(shapes), (set(sd) ^ set(shapes))
    for k, s in shapes.items():
        assert tuple(sd[k].shape) == tuple(s), (k, sd[k].shape, s)
        sd[k] = torch.from_numpy(fill_param(k, s))
    m.load_state_dict(sd)
    m.train()
    src, trg, meta = make_inputs(vocab, B, T, 568, 31)
    logits = m(torch.from_numpy(src), torch.from_numpy(meta))
    z = sh.train.filtered_logit(torch.from_numpy(src), logits)
    loss = torch.nn.CrossEntropyLoss()(z.reshape(-1, vocab.size), torch.from_numpy(trg).view(-1))
    loss.backward()
    out["src"], out["trg"], out["meta"] = src, trg, meta
    out["loss"] = np.array(loss.item(), dtype=np.float64)
    P = projection(vocab.size)
    out["logits_proj"] = (logits.detach() @ P).numpy()
    out["logits_rows"] = logits.detach()[:, [0, 149, T - 1], :].numpy()
    for k, p in m.named_parameters():
        gf = p.grad.reshape(-1).double()
        out[f"gsum:{k}"] = np.array([gf.sum().item(), gf.abs().sum().item(), (gf * gf).sum().item()])
        out[f"gpick:{k}"] = p.grad.reshape(-1)[:: max(1, gf.numel() // 64)][:64].numpy()
    np.savez_compressed(OUT / "g5_mamba.npz", **out)


if __name__ == "__main__":
    ref = Path(sys.argv[1] if len(sys.argv) > 1 else "/root/reference")
    torch.manual_seed(0)
    torch.set_num_threads(8)
    which = sys.argv[2] if len(sys.argv) > 2 else "all"
    if which in ("all", "g12"):
        g1_g2(ref)
    if which in ("all", "g3"):
        g3(ref)
    if which in ("all", "g4"):
        g4(ref)
    if which in ("all", "g5"):
        g5(ref)
    print("golden fixtures written to", OUT)

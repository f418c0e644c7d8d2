"""Diagnostic: relative-attention bf16 backward against the oracle, error per
gradient and per row region. Usage: python tools/attn_diag.py B S H"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import _pkgload  # noqa: E402

_pkgload.load()
import torch  # noqa: E402
from test_attention_gpu import _mk, _ref  # noqa: E402
from midiseq import attention as att  # noqa: E402

B, S, H = (int(x) for x in sys.argv[1:4])
hs = 128
scale = (H * hs) ** -0.5
qkv, R, dout = _mk(B, S, H, hs, S + 5, torch.bfloat16, seed=S)
ref_out, ref_dqkv, ref_dR = _ref(qkv, R, dout, B, S, H, hs, scale)
out, lse = att.relattn_fwd(qkv.cuda(), R.cuda(), B, S, H, hs, scale)
dqkv, dR = att.relattn_bwd(dout.cuda(), out, lse, qkv.cuda(), R.cuda(), B, S, H, hs, scale)
torch.cuda.synchronize()
nq = H * hs
tag = "kv5"


def rel(a, b):
    return ((a.float().cpu() - b).abs().max() / (b.abs().max() + 1e-12)).item()


print(f"kv{tag} B={B} S={S} H={H} out {rel(out, ref_out):.3e} dR {rel(dR[:, :S], ref_dR[:, :S]):.3e}")
dRe = (dR[:, :S].cpu() - ref_dR[:, :S]).abs().amax(dim=(0, 2)) / ref_dR[:, :S].abs().max()
print("  dR rows over 2e-2:", (dRe > 2e-2).nonzero().flatten().tolist()[:20])
for name, sl in (("dq", slice(0, nq)), ("dk", slice(nq, 2 * nq)), ("dv", slice(2 * nq, 3 * nq))):
    g = dqkv[:, sl].float().cpu().view(B, S, H, hs)
    r = ref_dqkv[:, sl].view(B, S, H, hs)
    mx = r.abs().max().item()
    rows = (g - r).abs().amax(dim=(0, 2, 3)) / mx
    bad = (rows > 2e-2).nonzero().flatten().tolist()
    print(f"  {name}: max {rows.max().item():.3e}  rows over 2e-2: {len(bad)} {bad[:24]}")

# metadata-prefix pairs i < j < 6 (keys every query sees): their dK contribution
qf = qkv.float().view(B, S, 3, H, hs)
Rf = R.float()
do = dout.float().view(B, S, H, hs)
O = ref_out.view(B, S, H, hs)
pair_dk = torch.zeros(B, 6, H, hs)
for b in range(B):
    for h in range(H):
        Lrow = None
        for i in range(5):
            # lse_i from the full reference row
            s_all = []
            for j in range(S):
                if j <= i or j < 6:
                    s = qf[b, i, 0, h] @ qf[b, j, 1, h]
                    if j <= i:
                        s = s + qf[b, i, 0, h] @ Rf[h, S - 1 - i + j]
                    elif j >= i + 2:
                        s = s + qf[b, i + 1, 0, h] @ Rf[h, j - i - 2]
                    s_all.append((j, s * scale))
            lse_i = torch.logsumexp(torch.stack([v for _, v in s_all]), 0)
            D = do[b, i, h] @ O[b, i, h]
            for j, sv in s_all:
                if j > i:
                    p = torch.exp(sv - lse_i)
                    ds = p * (do[b, i, h] @ qf[b, j, 2, h] - D) * scale
                    pair_dk[b, j, h] += ds * qf[b, i, 0, h]
g = dqkv[:, nq:2 * nq].float().cpu().view(B, S, H, hs)[:, :6]
r = ref_dqkv[:, nq:2 * nq].view(B, S, H, hs)[:, :6]
err = g - r
print("  dk rows 0-5: |err| %.3e  |pair| %.3e  |err+pair| %.3e  |err-pair| %.3e" % (
    err.abs().max(), pair_dk.abs().max(), (err + pair_dk).abs().max(), (err - pair_dk).abs().max()))

# the stored dS (r-indexed dQR, workspace head) against the reference dS
from midiseq import ops  # noqa: E402
ws = [v for k, v in ops._ws_cache.items() if k[0] == "attn"][0]
ldr = (S + 200 + 7) // 8 * 8
dqr = ws[: H * B * S * ldr * 2].view(torch.bfloat16).view(H, B, S, ldr).float().cpu()
Q, K, V = qf[:, :, 0], qf[:, :, 1], qf[:, :, 2]
for h in range(H):
    for b in range(B):
        q, k, v = Q[b, :, h], K[b, :, h], V[b, :, h]
        ac = q @ k.T
        bd = q @ Rf[h, :S].T  # [i][r]
        BDs = torch.zeros(S, S)
        for i in range(S):
            for j in range(S):
                if j <= i:
                    BDs[i, j] = bd[i, S - 1 - i + j]
                elif j >= i + 2:
                    BDs[i, j] = bd[i + 1, j - i - 2]
        sc = (ac + BDs) * scale
        ii, jj = torch.meshgrid(torch.arange(S), torch.arange(S), indexing="ij")
        allowed = (jj <= ii) | (jj < 6)
        sc = sc.masked_fill(~allowed, float("-inf"))
        P = torch.softmax(sc, -1)
        dP = do[b, :, h] @ v.T
        Dd = (do[b, :, h] * O[b, :, h]).sum(-1, keepdim=True)
        dS = P * (dP - Dd) * scale
        got = torch.zeros(S, S)
        for i in range(S):
            got[i, : i + 1] = dqr[h, b, i, S - 1 - i: S]
        ref = dS.tril()
        e = (got - ref).abs()
        mx = ref.abs().max()
        bad = (e > 2e-2 * mx).nonzero()
        print(f"  dS h{h} b{b}: max err {e.max() / mx:.3e}; bad entries {len(bad)}: {bad[:12].tolist()}")
        if h == 0 and b == 0:
            torch.set_printoptions(precision=4, linewidth=160)
            print("  got dS[0:7, 0:7]\n", got[:7, :7])
            print("  ref dS[0:7, 0:7]\n", ref[:7, :7])

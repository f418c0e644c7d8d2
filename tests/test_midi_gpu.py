"""Device token -> note decode (msq_midi_decode, csrc/midi.hip) against G7 (the
reference's own processing.decode) and the oracle (oracle/midi.py):
bit-exact note fields, beats and fp64 seconds, incl. a strided batch of
generate()-sized rows, rows without notes and the reference's errors."""
from pathlib import Path

import numpy as np
import pytest
import torch

from midiseq import midi
from oracle import midi as omidi
from oracle.fill import REAL, grammar_tokens

pytestmark = pytest.mark.gpu
G7 = np.load(Path(__file__).parent / "golden" / "g7_midi.npz")


def _check_row(nb, b, ref):
    n = int(nb.count[b])
    assert n == len(ref)
    f = torch.stack([nb.pitch[b, :n], nb.channel[b, :n], nb.dyn[b, :n], nb.tempo[b, :n]], 1).cpu().numpy()
    np.testing.assert_array_equal(f, np.array([r[:4] for r in ref]).reshape(-1, 4))
    np.testing.assert_array_equal(nb.beat_start[b, :n].cpu().numpy(), [r[4] for r in ref])
    np.testing.assert_array_equal(nb.beat_end[b, :n].cpu().numpy(), [r[5] for r in ref])
    np.testing.assert_array_equal(nb.t_start[b, :n].cpu().numpy(), np.array([r[6] for r in ref], dtype=np.float64))
    np.testing.assert_array_equal(nb.t_end[b, :n].cpu().numpy(), np.array([r[7] for r in ref], dtype=np.float64))


def test_decode_matches_reference_golden():
    toks = torch.from_numpy(G7["tokens"]).cuda()
    nb = midi.decode_batch(toks)
    torch.cuda.synchronize()
    for r in range(toks.shape[0]):
        ref_f, ref_t = G7[f"notes_{r}"], G7[f"times_{r}"]
        n = int(nb.count[r])
        assert n == len(ref_f)
        f = torch.stack([nb.pitch[r, :n], nb.channel[r, :n], nb.dyn[r, :n], nb.tempo[r, :n]], 1).cpu().numpy()
        np.testing.assert_array_equal(f, ref_f)
        np.testing.assert_array_equal(nb.t_start[r, :n].cpu().numpy(), ref_t[:, 0])
        np.testing.assert_array_equal(nb.t_end[r, :n].cpu().numpy(), ref_t[:, 1])
        # the per-row drop-in returns the reference's MIDI_note list
        notes = midi.decode(toks[r])
        assert [(x.pitch, x.channel, x.dynamic, x.tempo) for x in notes] == \
            [(v[0], v[1], v[2], float(v[3])) for v in ref_f.tolist()]
        assert [x.time_start for x in notes] == ref_t[:, 0].tolist()


@pytest.mark.parametrize("B,L", [(64, 4048), (3, 1), (5, 63), (2, 65), (3, 257), (2, 1000), (1, 15872)])
def test_decode_batch_matches_oracle(B, L):
    rng = np.random.default_rng(B * 1000 + L)
    s, V = REAL.start, REAL.size
    rows = np.stack([grammar_tokens(rng, REAL, L) for _ in range(B)])
    rows[rows >= s["tempo"]] = np.maximum(rows[rows >= s["tempo"]], s["tempo"] + 1)  # tempo > 0
    if B > 2:  # a shuffled row: arbitrary class order
        cls = rng.integers(0, 5, L)
        lo = np.array([0, s["dyn"], s["length"], s["time"], s["tempo"] + 1])
        hi = np.array([s["dyn"], s["length"], s["time"], s["tempo"], V])
        rows[1] = rng.integers(lo[cls], hi[cls])
    # strided rows (ld > L), as a slice of generate()'s output
    buf = torch.zeros(B, L + 7, dtype=torch.int64, device="cuda")
    buf[:, 3:3 + L] = torch.from_numpy(rows).cuda()
    nb = midi.decode_batch(buf[:, 3:3 + L])
    torch.cuda.synchronize()
    for b in range(B):
        try:
            ref = omidi.decode(rows[b], s)
        except IndexError:
            ref = []
        _check_row(nb, b, ref)


def test_decode_errors_like_reference():
    s = REAL.start
    with pytest.raises(IndexError):
        midi.decode([s["dyn"], s["length"], s["time"] + 3])
    with pytest.raises(ZeroDivisionError):
        midi.decode([5, s["dyn"], s["length"], s["tempo"], 6, s["dyn"], s["length"], s["tempo"] + 3])
    # a zero tempo on the LAST note is never a divisor: the reference decodes it
    notes = midi.decode([5, s["dyn"], s["length"], s["tempo"] + 9, 6, s["dyn"] + 1, s["length"] + 2, s["tempo"]])
    ref = omidi.decode([5, s["dyn"], s["length"], s["tempo"] + 9, 6, s["dyn"] + 1, s["length"] + 2, s["tempo"]], s)
    assert [(x.time_start, x.time_end) for x in notes] == [(r[6], r[7]) for r in ref]

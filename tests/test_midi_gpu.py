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


G8 = np.load(Path(__file__).parent / "golden" / "g8_encode.npz")


def _g8_notes(s):
    f, t = G8[f"notes_{s}"], G8[f"times_{s}"]
    return [midi.MIDI_note(pitch=int(a[0]), time_start=float(b[0]), time_end=float(b[1]), dynamic=int(a[2]),
                           channel=int(a[1]), tempo=int(a[3])) for a, b in zip(f, t)]


def test_encode_batch_matches_reference_golden():
    """msq_midi_encode over all G8 songs in one launch: tokens and adjusted
    beats bit-exact against the reference's processing.encode (G8)."""
    n = int(G8["n_songs"])
    toks, beats = midi.encode_batch([_g8_notes(s) for s in range(n)])
    for s in range(n):
        np.testing.assert_array_equal(beats[s], G8[f"beats_{s}"])
        np.testing.assert_array_equal(toks[s], G8[f"tokens_{s}"])


def test_encode_dropin_mutates_notes_like_reference():
    notes = _g8_notes(0)
    toks = midi.encode(notes)
    assert toks == G8["tokens_0"].tolist()
    assert [(n.time_start, n.time_end) for n in notes] == [tuple(b) for b in G8["beats_0"].tolist()]


def test_encode_large_batch_against_oracle():
    """Many long songs (several 64-note steps, carries across steps) against
    the oracle; then decode_batch of the encoded rows gives back the notes."""
    rng = np.random.default_rng(11)
    songs = []
    for s in range(40):
        n = int(rng.integers(1, 3000))
        t = np.cumsum(rng.choice([0.0, 0.02, 0.3, 1.0], size=n))
        tp = rng.integers(30, 240, size=n)
        songs.append([midi.MIDI_note(pitch=int(rng.integers(0, 128)), time_start=float(t[k]),
                                     time_end=float(t[k] + rng.random() * 2), dynamic=int(rng.integers(1, 128)),
                                     channel=int(rng.integers(0, 128)), tempo=int(tp[k])) for k in range(n)])
    toks, beats = midi.encode_batch(songs)
    for s, notes in enumerate(songs):
        rows = [[m.pitch, m.channel, m.dynamic, m.tempo, m.time_start, m.time_end] for m in notes]
        np.testing.assert_array_equal(beats[s], np.array(omidi.adjust_note_time(rows)))
        np.testing.assert_array_equal(toks[s], np.array(omidi.encode(rows, REAL.start)))
    nb = midi.decode_batch(torch.from_numpy(toks[3]).cuda())
    assert int(nb.count[0]) == len(songs[3])
    np.testing.assert_array_equal(nb.pitch[0, :len(songs[3])].cpu().numpy(), [m.pitch for m in songs[3]])


def test_extract_encode_from_smf_file(tmp_path):
    """extract_midi over a file written by midiseq.smf: the notes come back
    (parity of extraction vs pretty_midi is unpinned; the round trip is the
    check), then preprocess_midi_files writes the token row."""
    from midiseq import smf
    rng = np.random.default_rng(3)
    notes = []
    t = 0.0
    for k in range(250):
        t += float(rng.choice([0.0, 0.25, 0.5]))
        notes.append(midi.MIDI_note(pitch=int(rng.integers(30, 90)), time_start=t, time_end=t + 0.25,
                                    dynamic=int(rng.integers(20, 120)), channel=int(rng.integers(0, 3)), tempo=120.0))
    src = tmp_path / "midi" / "model" / "Mozart" / "song.mid"
    src.parent.mkdir(parents=True)
    smf.note_to_midi(notes, str(src))
    back = midi.extract_midi(str(src))
    assert len(back) == len(set(notes))
    assert all(n.tempo == 120 for n in back)
    out = midi.preprocess_midi_files(str(tmp_path / "midi"), str(tmp_path / "npy"))
    assert len(out) == 1 and out[0].endswith("model/Mozart/song.npy")
    row = np.load(out[0])
    assert row.dtype == np.int64 and len(row) >= 4 * len(back)

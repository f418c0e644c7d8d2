"""Oracle token -> note decode (oracle/midi.py) against G7, the reference's own
processing.decode run on the same rows (tests/golden/make_g7_midi.py):
bit-exact note fields and fp64 times."""
from pathlib import Path

import numpy as np
import pytest

from oracle import midi as omidi
from oracle.fill import REAL

G7 = np.load(Path(__file__).parent / "golden" / "g7_midi.npz")


@pytest.mark.parametrize("r", range(G7["tokens"].shape[0]))
def test_oracle_decode_matches_reference(r):
    notes = omidi.decode(G7["tokens"][r], REAL.start)
    ref_f, ref_t = G7[f"notes_{r}"], G7[f"times_{r}"]
    assert len(notes) == len(ref_f) > 0
    got_f = np.array([[n[0], n[1], n[2], n[3]] for n in notes])
    got_t = np.array([[n[6], n[7]] for n in notes])
    np.testing.assert_array_equal(got_f, ref_f)
    np.testing.assert_array_equal(got_t, ref_t)  # bit-identical doubles


def test_oracle_decode_errors_like_reference():
    s = REAL.start
    with pytest.raises(IndexError):  # no complete note: revert_note_time reads notes[0]
        omidi.decode([s["dyn"], s["length"]], s)
    with pytest.raises(ZeroDivisionError):  # tempo token 0 -> 60 / 0.0
        omidi.decode([5, s["dyn"], s["length"], s["tempo"], 6, s["dyn"], s["length"], s["tempo"] + 3], s)


G8 = np.load(Path(__file__).parent / "golden" / "g8_encode.npz")


def g8_song(s):
    f, t = G8[f"notes_{s}"], G8[f"times_{s}"]
    return [[int(a[0]), int(a[1]), int(a[2]), int(a[3]), float(b[0]), float(b[1])] for a, b in zip(f, t)]


@pytest.mark.parametrize("s", range(int(G8["n_songs"])))
def test_oracle_encode_matches_reference(s):
    """note -> token encode (processing.py:111-152) against G8: the adjusted
    integer beats and the token list, bit-exact (clamps, repeated time
    shifts, zero-length notes included)."""
    notes = g8_song(s)
    np.testing.assert_array_equal(np.array(omidi.adjust_note_time(notes)), G8[f"beats_{s}"])
    np.testing.assert_array_equal(np.array(omidi.encode(notes, REAL.start)), G8[f"tokens_{s}"])


def test_encode_decode_round_trip_structure():
    """decode(encode(notes)) gives back every note's pitch / channel / dyn /
    tempo and its beat grid up to the length clamp (511 beats), while no time
    shift was clamped — the codec's own invariant."""
    notes = g8_song(0)
    toks = omidi.encode(notes, REAL.start)
    back = omidi.decode(toks, REAL.start)
    beats = omidi.adjust_note_time(notes)
    assert len(back) == len(notes)
    prev = 0
    for n, b, (bs, be) in zip(notes, back, beats):
        assert (b[0], b[1], b[2], b[3]) == (n[0], n[1], n[2], n[3])
        assert bs - prev < 511 and b[4] == bs and b[5] - b[4] == min(be - bs, 511)
        prev = bs

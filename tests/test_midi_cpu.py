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

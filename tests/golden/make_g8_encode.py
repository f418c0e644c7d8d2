"""G8 golden vectors for the note -> token encode, from the REFERENCE's own
processing/processing.py ``encode`` (+ ``adjust_note_time``, :111-152) run in
the build container through the test-only shim of make_golden.py (pretty_midi
stubbed: encode does not use it). The reference never travels; only the
vectors do.

Run:  python tests/golden/make_g8_encode.py [/root/reference]

Songs (lists of the reference's MIDI_note, sorted by time_start as
extract_midi leaves them, seconds as floats, integer tempos as round(bpm)):
  * realistic songs: chords (equal starts), tempo changes, short and long notes;
  * clamp cases: pitch + channel*128 past the pitch block, velocity >= 128,
    lengths and time shifts past 511 beats, tempo >= 250;
  * zero-length notes (time_end == time_start -> one beat) and a 1-note song.
Stored per song s: the six note columns (input), the adjusted beats
(time_start / time_end after adjust_note_time) and the token list."""
import sys
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(REPO / "tests" / "golden"))
sys.path.insert(0, str(REPO))
from make_golden import RefShim  # noqa: E402
from oracle.fill import REAL  # noqa: E402

OUT = REPO / "tests" / "golden" / "g8_encode.npz"


def songs():
    rng = np.random.default_rng(8)
    out = []
    for s in range(6):
        n = int(rng.integers(50, 400))
        t, rows = 0.0, []
        tempo = int(rng.integers(40, 200))
        for _ in range(n):
            if rng.random() < 0.3:  # chord: same start as the previous note
                dt = 0.0
            else:
                dt = float(rng.choice([rng.random() * 0.5, rng.random() * 0.05, rng.random() * 3.0]))
            t += dt
            if rng.random() < 0.05:
                tempo = int(rng.integers(40, 200))
            dur = float(rng.choice([rng.random() * 0.01, rng.random() * 0.8, rng.random() * 6.0]))
            rows.append((int(rng.integers(0, 128)), t, t + dur, int(rng.integers(1, 128)), int(rng.integers(0, 128)),
                         tempo))
        out.append(rows)
    # clamp cases
    rows, t = [], 0.0
    for k in range(120):
        t += float(rng.choice([0.0, 0.1, 40.0, 400.0]))
        rows.append((int(rng.integers(0, 128)), t, t + float(rng.choice([0.0, 0.2, 90.0])),
                     int(rng.choice([5, 127, 128, 200])), int(rng.choice([0, 127, 128, 140])),
                     int(rng.choice([10, 120, 249, 250, 300]))))
    out.append(rows)
    out.append([(60, 0.25, 0.25, 90, 0, 120)])  # one zero-length note
    return out


def main(ref=Path(sys.argv[1] if len(sys.argv) > 1 else "/root/reference")):
    sh = RefShim(ref, REAL, 568)
    sys.path.insert(0, str(ref))
    note = sh._load("note", "note.py")
    proc = sh._load("ref_processing", "processing/processing.py")
    res = {}
    for s, rows in enumerate(songs()):
        res[f"notes_{s}"] = np.array([[p, ch, dy, tp] for p, _, _, dy, ch, tp in rows], dtype=np.int64)
        res[f"times_{s}"] = np.array([[a, b] for _, a, b, _, _, _ in rows], dtype=np.float64)
        notes = [note.MIDI_note(pitch=p, time_start=a, time_end=b, dynamic=dy, channel=ch, tempo=tp)
                 for p, a, b, dy, ch, tp in rows]
        toks = proc.encode(notes)
        res[f"tokens_{s}"] = np.array(toks, dtype=np.int64)
        res[f"beats_{s}"] = np.array([[n.time_start, n.time_end] for n in notes], dtype=np.int64)
    res["n_songs"] = np.array(len(songs()))
    np.savez_compressed(OUT, **res)
    print("wrote", OUT, {k: v.shape for k, v in res.items() if k.endswith("_0")})


if __name__ == "__main__":
    main()

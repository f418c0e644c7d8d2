"""G7 golden vectors for the token -> note decode, from the REFERENCE's own
processing/processing.py ``decode`` (+ ``revert_note_time``) run in the build
container through the test-only shim of make_golden.py (pretty_midi stubbed:
decode does not use it). The reference never travels; only the vectors do.

Run:  python tests/golden/make_g7_midi.py [/root/reference]

Rows (real vocabulary, config.yaml discretization, bar_res 64):
  * grammar-cycled rows (SURVEY.md §8(d) cycle, optional time shifts);
  * shuffled rows (random class order: partial notes, repeated fields,
    the field-reset rule, time shifts that persist across notes);
  * edge tokens (first/last token of every class, channel > 0, drums 128).
Stored: tokens [R, L] int64, and per row the note fields and fp64 times.
"""
import sys
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(REPO / "tests" / "golden"))
sys.path.insert(0, str(REPO))
from make_golden import RefShim  # noqa: E402
from oracle.fill import REAL, grammar_tokens  # noqa: E402

OUT = REPO / "tests" / "golden" / "g7_midi.npz"


def rows(L=300):
    rng = np.random.default_rng(7)
    s, V = REAL.start, REAL.size
    out = [grammar_tokens(rng, REAL, L) for _ in range(3)]
    for _ in range(3):  # random class order, tempo > 0 so revert_note_time is defined
        cls = rng.integers(0, 5, L)
        lo = np.array([s["pitch"], s["dyn"], s["length"], s["time"], s["tempo"] + 1])
        hi = np.array([s["dyn"], s["length"], s["time"], s["tempo"], V])
        out.append(rng.integers(lo[cls], hi[cls]))
    edge = []
    ends = [(s["pitch"], s["dyn"] - 1), (s["dyn"], s["length"] - 1), (s["length"], s["time"] - 1),
            (s["time"], s["tempo"] - 1), (s["tempo"] + 1, V - 1)]
    while len(edge) < L:
        for c, (a, b) in enumerate(ends):
            if c == 0:
                edge.append(int(rng.choice([a, b, 128 * 128 + 5, 128 * 3 + 60])))
            else:
                edge.append(int(rng.choice([a, b])))
    out.append(np.asarray(edge[:L]))
    return np.stack(out).astype(np.int64)


def main(ref=Path(sys.argv[1] if len(sys.argv) > 1 else "/root/reference")):
    sh = RefShim(ref, REAL, 568)
    sys.path.insert(0, str(ref))
    sh._load("note", "note.py")
    proc = sh._load("ref_processing", "processing/processing.py")
    toks = rows()
    res = {"tokens": toks}
    for r, row in enumerate(toks):
        notes = proc.decode(list(int(t) for t in row))
        res[f"notes_{r}"] = np.array([[n.pitch, n.channel, n.dynamic, n.tempo] for n in notes], dtype=np.int64)
        res[f"times_{r}"] = np.array([[n.time_start, n.time_end] for n in notes], dtype=np.float64)
    np.savez_compressed(OUT, **res)
    print("wrote", OUT, {k: v.shape for k, v in res.items() if k.startswith(("tokens", "notes_0"))})


if __name__ == "__main__":
    main()

"""TEST INFRASTRUCTURE ONLY — CPU restatement of the reference's token -> note
decode (processing/processing.py:171-214 ``decode``) and its beat -> seconds
step (:154-169 ``revert_note_time``). Imported by tests/ only, as the checker
of the device path (midiseq.midi / csrc/midi.hip). Pinned by G7
(tests/golden/g7_midi.npz, made by running the reference's own decode).

Pure-Python loops, in the reference's operation order, so the fp64 note times
are bit-identical to the reference's.
"""


def decode(tokens, start, disc_pitch=128, res_per_beat=64):
    """tokens: iterable of ints; start: dict of class start indices
    (configs/common/__init__.py start_idx). Returns a list of
    (pitch, channel, dyn, tempo, beat_start, beat_end, t_start, t_end).
    Raises IndexError on a row without notes and ZeroDivisionError on a zero
    tempo where the reference does (revert_note_time)."""
    notes = []
    prev_time = 0
    dyn = pitch = length = channel = tempo = None
    time_delta = 0
    for tok in tokens:  # processing.py:182-209
        tok = int(tok)
        if tok < start["dyn"]:
            channel, pitch = divmod(tok, disc_pitch)
        elif tok < start["length"]:
            dyn = tok - start["dyn"]
        elif tok < start["time"]:
            length = tok - start["length"]
        elif tok < start["tempo"]:
            time_delta = tok - start["time"]
        else:
            tempo = tok - start["tempo"]
        if None not in (dyn, pitch, length, channel, tempo):
            bs = prev_time + time_delta
            notes.append([pitch, channel, dyn, tempo, bs, bs + length])
            dyn = pitch = length = channel = tempo = None
            prev_time = prev_time + time_delta
    # revert_note_time (processing.py:154-169)
    prev_tempo = float(notes[0][3])  # IndexError on an empty row, as the reference
    prev_t, prev_beat = 0, 0
    out = []
    for n in notes:
        resolution = 60 / prev_tempo / res_per_beat
        ts = prev_t + (float(n[4]) - prev_beat) * resolution
        te = ts + (float(n[5]) - float(n[4])) * resolution
        prev_t, prev_beat, prev_tempo = ts, float(n[4]), float(n[3])
        out.append((n[0], n[1], n[2], n[3], n[4], n[5], ts, te))
    return out

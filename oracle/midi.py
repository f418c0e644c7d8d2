"""TEST INFRASTRUCTURE ONLY — CPU restatement of the reference's note <-> token
codec: the token -> note decode (processing/processing.py:171-214 ``decode``)
with its beat -> seconds step (:154-169 ``revert_note_time``), and the note ->
token encode (:129-152 ``encode``) with its seconds -> beats step (:111-126
``adjust_note_time``). Imported by tests/ only, as the checker of the device
path (midiseq.midi / csrc/midi.hip). Pinned by G7 / G8 (tests/golden/
g7_midi.npz, g8_encode.npz: the reference's own decode / encode).

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


def adjust_note_time(notes, res_per_beat=64):
    """processing.py:111-126: note seconds -> integer beats, in the reference's
    operation order (fp64 running sum of (start - prev_start) / resolution,
    resolution from the PREVIOUS note's tempo; int() truncation; a note whose
    end truncates to its start lasts one beat). notes: list of
    [pitch, channel, dyn, tempo, t_start, t_end]; returns [(beat_start, beat_end)]."""
    cur, prev_time, prev_tempo = 0, 0, notes[0][3]
    out = []
    for n in notes:
        resolution = 60 / prev_tempo / res_per_beat
        cur += (n[4] - prev_time) / resolution
        fut = cur + (n[5] - n[4]) / resolution
        prev_time, prev_tempo = n[4], n[3]
        bs = int(cur)
        out.append((bs, bs + 1 if int(fut) == int(cur) else int(fut)))
    return out


def encode(notes, start, disc=(128, 129, 128, 512, 512, 250), res_per_beat=64):
    """processing.py:129-152: notes -> token ids (pitch, dyn, length, time shift
    only when it changes, tempo), with the reference's clamps."""
    P, C, D, Ln, Tm, Tp = disc
    toks, time_prev, td_prev = [], 0, 0
    for n, (bs, be) in zip(notes, adjust_note_time(notes, res_per_beat)):
        pitch, channel, dyn, tempo = n[0], n[1], n[2], n[3]
        td = start["time"] + min(bs - time_prev, Tm - 1)
        toks += [start["pitch"] + min(pitch + channel * P, P * C - 1), start["dyn"] + min(dyn, D - 1),
                 start["length"] + min(be - bs, Ln - 1)]
        if td_prev != td:
            toks.append(td)
        toks.append(start["tempo"] + min(tempo, Tp - 1))
        time_prev, td_prev = bs, td
    return toks

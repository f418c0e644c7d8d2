"""Standard MIDI File writer/reader for decoded notes (the step after
``midiseq.midi.decode``): drop-in for ``processing.note_to_midi(midi_notes,
output_path)`` (processing/processing.py:85-109, + ``update_tempo`` :216-225).

The reference writes through ``pretty_midi`` (absent from this image), so the
byte layout is this module's own and its output is NOT pinned to the
reference's; what it keeps from the reference is the musical content:

* one instrument track per note channel, in first-appearance order; channel
  >= 128 is a drum track (program channel - 128) (processing.py:88-105);
* a tempo event wherever the note tempo changes, at that note's start
  (update_tempo :216-224), default 120 bpm before the first one;
* note on/off at the decoded start/end seconds, converted to ticks through
  that tempo map at ``resolution`` ticks per beat (pretty_midi's default 220).

Host file I/O (not a device path): a few thousand notes per piece.
"""
import struct

DEFAULT_RESOLUTION = 220  # pretty_midi.PrettyMIDI() default ticks per beat
DEFAULT_BPM = 120.0


def _vlq(n):
    out = [n & 0x7F]
    n >>= 7
    while n:
        out.append(0x80 | (n & 0x7F))
        n >>= 7
    return bytes(reversed(out))


def _tempo_map(notes):
    """[(time_s, bpm)] per update_tempo: a change wherever note.tempo differs
    from the previous change (first note always, since prev starts at 0)."""
    changes, prev = [], 0
    for n in notes:
        if n.tempo != prev:
            changes.append((float(n.time_start), float(n.tempo)))
            prev = n.tempo
    if not changes or changes[0][0] > 0.0:
        changes.insert(0, (0.0, DEFAULT_BPM))
    # keep the last change at any given time, in time order
    out = []
    for t, bpm in sorted(changes, key=lambda c: c[0]):
        if out and out[-1][0] == t:
            out[-1] = (t, bpm)
        else:
            out.append((t, bpm))
    return out


def _seconds_to_ticks(tmap, resolution):
    """Returns (tick_of(t), [(tick, bpm)]) for a piecewise-constant tempo map."""
    seg = []  # (t0, tick0, seconds per tick)
    tick0 = 0.0
    for i, (t, bpm) in enumerate(tmap):
        if i:
            pt, ptick, spt = seg[-1]
            tick0 = ptick + (t - pt) / spt
        seg.append((t, tick0, 60.0 / (bpm * resolution)))

    def tick_of(t):
        k = len(seg) - 1
        while k > 0 and seg[k][0] > t:
            k -= 1
        t0, tk, spt = seg[k]
        return int(round(tk + (t - t0) / spt))
    return tick_of, [(int(round(tk)), bpm) for (t0, tk, _), (_, bpm) in zip(seg, tmap)]


def _track(events):
    """events: [(tick, order, bytes)] -> MTrk chunk with delta times."""
    body, last = bytearray(), 0
    for tick, _, msg in sorted(events, key=lambda e: (e[0], e[1])):
        body += _vlq(tick - last) + msg
        last = tick
    body += _vlq(0) + b"\xff\x2f\x00"
    return b"MTrk" + struct.pack(">I", len(body)) + bytes(body)


def note_to_midi(midi_notes, output_path, resolution=DEFAULT_RESOLUTION):
    """processing.note_to_midi drop-in: list of MIDI_note (seconds) -> .mid file."""
    tick_of, tempo_ticks = _seconds_to_ticks(_tempo_map(midi_notes), resolution)
    tracks = []
    tempo_ev = []
    for tick, bpm in tempo_ticks:
        us = max(1, min(0xFFFFFF, int(round(60_000_000 / bpm)))) if bpm > 0 else 0xFFFFFF
        tempo_ev.append((tick, 0, b"\xff\x51\x03" + us.to_bytes(3, "big")))
    tracks.append(_track(tempo_ev))
    by_channel = {}
    for n in midi_notes:  # processing.py:88-90, dict keeps first-appearance order
        by_channel.setdefault(n.channel, []).append(n)
    free = [c for c in range(16) if c != 9]
    for i, (channel, notes) in enumerate(by_channel.items()):
        drum = channel >= 128
        program = (channel - 128 if drum else channel) & 0x7F
        ch = 9 if drum else free[i % len(free)]
        ev = [(0, 0, bytes([0xC0 | ch, program]))]
        for n in notes:
            on, off = tick_of(float(n.time_start)), tick_of(float(n.time_end))
            p, v = int(n.pitch) & 0x7F, max(0, min(127, int(n.dynamic)))
            if v == 0:  # silent; a velocity-0 note-on would end another note of this pitch
                continue
            ev.append((max(off, on + 1), 1, bytes([0x80 | ch, p, 0])))  # no zero-length (stuck) notes
            ev.append((on, 2, bytes([0x90 | ch, p, v])))
        tracks.append(_track(ev))
    with open(output_path, "wb") as f:
        f.write(b"MThd" + struct.pack(">IHHH", 6, 1, len(tracks), resolution))
        for t in tracks:
            f.write(t)


def read_midi(path):
    """Minimal SMF reader (format 0/1, PPQ): -> (notes, tempos) with notes as
    (pitch, start_s, end_s, velocity, program, is_drum) sorted by start and
    tempos as [(time_s, bpm)]. Used for round trips and for reading MIDI files."""
    data = open(path, "rb").read()
    assert data[:4] == b"MThd", "not a MIDI file"
    hlen, fmt, ntrk, div = struct.unpack(">IHHH", data[4:14])
    assert not div & 0x8000, "SMPTE time division is not supported"
    pos, raw = 8 + hlen, []
    tempo_ticks = []
    for _ in range(ntrk):
        assert data[pos:pos + 4] == b"MTrk"
        ln = struct.unpack(">I", data[pos + 4:pos + 8])[0]
        trk, pos = data[pos + 8:pos + 8 + ln], pos + 8 + ln
        i, tick, status, program = 0, 0, 0, 0
        open_notes = {}
        while i < len(trk):
            d = 0
            while True:
                b = trk[i]
                i += 1
                d = (d << 7) | (b & 0x7F)
                if not b & 0x80:
                    break
            tick += d
            if trk[i] & 0x80:
                status = trk[i]
                i += 1
            if status == 0xFF:
                typ = trk[i]
                i += 1
                ln2 = 0
                while True:
                    b = trk[i]
                    i += 1
                    ln2 = (ln2 << 7) | (b & 0x7F)
                    if not b & 0x80:
                        break
                if typ == 0x51:
                    tempo_ticks.append((tick, int.from_bytes(trk[i:i + 3], "big")))
                i += ln2
                if typ == 0x2F:
                    break
                continue
            if status in (0xF0, 0xF7):
                ln2 = 0
                while True:
                    b = trk[i]
                    i += 1
                    ln2 = (ln2 << 7) | (b & 0x7F)
                    if not b & 0x80:
                        break
                i += ln2
                continue
            kind, ch = status & 0xF0, status & 0x0F
            nb = 1 if kind in (0xC0, 0xD0) else 2
            a = trk[i:i + nb]
            i += nb
            if kind == 0xC0:
                program = a[0]
            elif kind == 0x90 and a[1] > 0:
                open_notes.setdefault((ch, a[0]), []).append((tick, a[1]))
            elif kind == 0x80 or (kind == 0x90 and a[1] == 0):
                if open_notes.get((ch, a[0])):
                    t0, vel = open_notes[(ch, a[0])].pop(0)
                    raw.append((a[0], t0, tick, vel, program, ch == 9))
    tempo_ticks.sort(key=lambda e: e[0])  # stable: the later of two events at one tick wins
    if not tempo_ticks or tempo_ticks[0][0] > 0:
        tempo_ticks.insert(0, (0, 500000))
    seg, t = [], 0.0
    for k, (tk, us) in enumerate(tempo_ticks):
        if k:
            ptk, pus, pt = seg[-1]
            t = pt + (tk - ptk) * pus / 1e6 / div
        seg.append((tk, us, t))

    def sec(tick):
        k = len(seg) - 1
        while k > 0 and seg[k][0] > tick:
            k -= 1
        tk, us, t0 = seg[k]
        return t0 + (tick - tk) * us / 1e6 / div
    notes = sorted((p, sec(a), sec(b), v, prog, dr) for p, a, b, v, prog, dr in raw)
    notes.sort(key=lambda n: (n[1], n[0]))
    return notes, [(s[2], 60e6 / s[1]) for s in seg]

"""MIDI file writer (midiseq.smf.note_to_midi, drop-in for processing.note_to_midi
processing.py:85-109 + update_tempo :216-225). The reference writes through
pretty_midi, absent here, so byte-level parity is UNPINNED; these tests pin the
musical content: notes decoded from the G7 rows (the reference's own decode
output) survive write -> read within half a tick, tracks follow the channels
in first-appearance order, tempo events follow update_tempo."""
from pathlib import Path

import numpy as np
import pytest

from midiseq import smf
from midiseq.midi import MIDI_note
from oracle import midi as omidi
from oracle.fill import REAL

G7 = np.load(Path(__file__).parent / "golden" / "g7_midi.npz")
REF_MIDI = Path("/root/reference/scripts/midi")


def _notes(r):
    """Row r of G7 decoded by the oracle (bit-identical to the reference's
    decode, test_midi_cpu.py), with tempos below 4 bpm raised by 4: SMF tempo
    events cannot express less than 60e6 / 0xFFFFFF = 3.58 bpm."""
    toks = G7["tokens"][r].copy()
    t0 = REAL.start["tempo"]
    toks[(toks >= t0) & (toks < t0 + 4)] += 4
    return [MIDI_note(pitch=n[0], time_start=n[6], time_end=n[7], dynamic=n[2], channel=n[1], tempo=float(n[3]))
            for n in omidi.decode(toks, REAL.start)]


@pytest.mark.parametrize("r", range(G7["tokens"].shape[0]))
def test_round_trip_of_decoded_rows(tmp_path, r):
    notes = _notes(r)
    path = tmp_path / "x.mid"
    smf.note_to_midi(notes, path)
    back, tempos = smf.read_midi(path)
    # overlapping notes of one pitch pair up first-in-first-out in any MIDI
    # reader, so starts and ends are compared as per-pitch multisets
    tick_s = max(60.0 / (n.tempo * smf.DEFAULT_RESOLUTION) for n in notes if n.tempo > 0)
    sounding = [n for n in notes if n.dynamic > 0]  # a velocity-0 note-on IS a note-off in MIDI
    assert len(back) == len(sounding)
    for key in (1, 2):
        w = sorted((n.pitch, n.dynamic if key == 1 else 0, n.time_start if key == 1 else n.time_end)
                   for n in sounding)
        g = sorted((x[0], x[3] if key == 1 else 0, x[key]) for x in back)
        assert [x[:2] for x in w] == [x[:2] for x in g]
        # tempo events sit on whole ticks: per-change rounding accumulates over long pieces
        np.testing.assert_allclose([x[2] for x in g], [x[2] for x in w], atol=2 * tick_s, rtol=2e-4)
    # channels -> tracks in first-appearance order; drums (channel >= 128) on MIDI channel 9
    progs = {(prog, drum) for *_, prog, drum in back}
    chans = {(n.channel - 128 if n.channel >= 128 else n.channel, n.channel >= 128) for n in notes}
    assert progs <= chans
    # update_tempo: one tempo event per change of note tempo (at that note's start)
    changes = []
    for n in notes:
        if not changes or changes[-1][1] != n.tempo:
            if changes and changes[-1][0] == n.time_start:
                changes[-1] = (n.time_start, n.tempo)  # several changes at one instant: the last sets the tempo
            else:
                changes.append((n.time_start, n.tempo))
    got = tempos[1:] if changes[0][0] > 0 else tempos  # 120 bpm default before a first change after 0
    assert len(got) == len(changes)
    for (t, bpm), (gt, gb) in zip(changes, got):
        assert abs(gb - bpm) <= 1e-3 * bpm and abs(gt - t) <= 2 * tick_s * len(changes)


def test_header_and_tracks(tmp_path):
    notes = [MIDI_note(60, 0.0, 0.5, 100, 0, 120.0), MIDI_note(62, 0.5, 1.0, 90, 130, 120.0),
             MIDI_note(64, 1.0, 2.0, 80, 0, 60.0)]
    path = tmp_path / "y.mid"
    smf.note_to_midi(notes, path)
    data = path.read_bytes()
    assert data[:4] == b"MThd" and data[8:10] == b"\x00\x01"
    assert int.from_bytes(data[10:12], "big") == 3  # tempo track + 2 channels
    assert int.from_bytes(data[12:14], "big") == 220
    back, tempos = smf.read_midi(path)
    assert [(p, round(a, 6), round(b, 6), v, prog, d) for p, a, b, v, prog, d in back] == [
        (60, 0.0, 0.5, 100, 0, False), (62, 0.5, 1.0, 90, 2, True), (64, 1.0, 2.0, 80, 0, False)]
    assert [(round(t, 6), round(b, 6)) for t, b in tempos] == [(0.0, 120.0), (1.0, 60.0)]


@pytest.mark.skipif(not REF_MIDI.is_dir(), reason="reference MIDI files not mounted")
def test_reads_reference_midi_files():
    """The reference's own generated .mid files (written by pretty_midi) parse:
    notes with positive durations, valid pitches/velocities."""
    files = sorted(REF_MIDI.glob("*.mid"))
    assert files
    for f in files:
        notes, tempos = smf.read_midi(f)
        assert notes and tempos
        for p, a, b, v, prog, drum in notes:
            assert 0 <= p < 128 and 0 < v < 128 and b >= a >= 0

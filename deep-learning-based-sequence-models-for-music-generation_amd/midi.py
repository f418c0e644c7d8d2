"""The note <-> token codec on the device.

* Decode: drop-in for ``processing.decode(token_seq)`` (processing/processing.py
  :171-214, with revert_note_time :154-169) as called by scripts/
  generate_midi_combined.py:143-156 on each generated row. ``decode_batch``
  runs ONE launch of ``msq_midi_decode`` (csrc/midi.hip) over all B rows while
  they are still in HBM; ``decode`` returns the reference's list of
  ``MIDI_note`` for one row.
* Encode: drop-in for ``processing.encode(midi_notes)`` (:129-152, with
  adjust_note_time :111-126): ``encode_batch`` turns many songs' notes into
  token rows in ONE launch of ``msq_midi_encode``; ``extract_midi`` (:57-83)
  reads a .mid file through midiseq.smf (pretty_midi is absent here: parity
  of extraction itself is unpinned) and ``preprocess_midi_files`` (:24-55)
  writes the ``<out>/<model>/<band>/<song>.npy`` token store the data feed
  loads.

No CPU fallback: without libmidiseq.so the call raises RuntimeError.
"""
import ctypes
from dataclasses import dataclass

import torch

from ._lib import call, ptr, stream
from .config import DEFAULT_DISC, Discretization

BAR_RES = 64  # config.yaml resolution.bar_res
MAX_ROW = 256 * 62  # msq_midi_decode row limit (staged in 64 KB of LDS)


class MIDI_note:
    """Same fields and equality as the reference's note.py:1-28."""

    def __init__(self, pitch, time_start, time_end, dynamic, channel, tempo):
        self.pitch, self.time_start, self.time_end = pitch, time_start, time_end
        self.dynamic, self.channel, self.tempo = dynamic, channel, tempo

    def __repr__(self):
        return (f"MIDI_note(pitch={self.pitch}, time_start={self.time_start}, "
                f"time_end={self.time_end}, dynamic={self.dynamic}, channel={self.channel}, tempo={self.tempo})")

    def __eq__(self, other):
        return isinstance(other, MIDI_note) and (self.pitch, self.time_start, self.time_end, self.dynamic,
                                                 self.channel) == (other.pitch, other.time_start, other.time_end,
                                                                   other.dynamic, other.channel)

    def __hash__(self):
        return hash((self.pitch, self.time_start, self.time_end, self.dynamic, self.channel))

    def note2seq(self):
        return [self.dynamic, self.pitch, self.time_end - self.time_start]


@dataclass
class NoteBatch:
    """Device-resident decode of B rows: row b's notes are [b, :count[b]]."""
    pitch: torch.Tensor       # int32 [B, cap]
    channel: torch.Tensor     # int32 [B, cap]
    dyn: torch.Tensor         # int32 [B, cap]
    tempo: torch.Tensor       # int32 [B, cap]
    beat_start: torch.Tensor  # int64 [B, cap]  (note time in beats, before revert_note_time)
    beat_end: torch.Tensor    # int64 [B, cap]
    t_start: torch.Tensor     # float64 [B, cap] seconds
    t_end: torch.Tensor       # float64 [B, cap]
    count: torch.Tensor       # int64 [B]

    def notes(self, b):
        """Row b as the reference's list of MIDI_note (host copy of one row),
        raising where the reference's decode raises."""
        n = int(self.count[b])
        if n == 0:  # revert_note_time reads midi_notes[0] (processing.py:158)
            raise IndexError("list index out of range")
        cols = [t[b, :n].cpu().tolist() for t in (self.pitch, self.channel, self.dyn, self.tempo,
                                                  self.t_start, self.t_end)]
        tempos = cols[3]
        if tempos[0] == 0 or 0 in tempos[:-1]:  # 60 / prev_tempo (processing.py:160)
            raise ZeroDivisionError("float division by zero")
        return [MIDI_note(pitch=p, time_start=ts, time_end=te, dynamic=d, channel=c, tempo=float(tp))
                for p, c, d, tp, ts, te in zip(*cols)]


def decode_batch(rows: torch.Tensor, disc: Discretization = DEFAULT_DISC, res_per_beat: int = BAR_RES,
                 out: NoteBatch = None) -> NoteBatch:
    """rows: int64 [B, L] (or [L]) token ids on the GPU -> NoteBatch (one launch)."""
    if rows.dim() == 1:
        rows = rows[None]
    if rows.dtype != torch.int64 or not rows.is_cuda or rows.stride(1) != 1:
        raise ValueError("decode_batch: rows must be a row-contiguous int64 CUDA tensor")
    B, L = rows.shape
    if L > MAX_ROW:
        raise ValueError(f"decode_batch: rows longer than {MAX_ROW} tokens")
    cap = L // 4 + 1  # a note takes at least 4 tokens (pitch, dyn, length, tempo)
    if out is None:
        dev = rows.device
        i32 = dict(dtype=torch.int32, device=dev)
        out = NoteBatch(*(torch.empty(B, cap, **i32) for _ in range(4)),
                        torch.empty(B, cap, dtype=torch.int64, device=dev),
                        torch.empty(B, cap, dtype=torch.int64, device=dev),
                        torch.empty(B, cap, dtype=torch.float64, device=dev),
                        torch.empty(B, cap, dtype=torch.float64, device=dev),
                        torch.empty(B, dtype=torch.int64, device=dev))
    d = (ctypes.c_int64 * 6)(disc.pitch, disc.channel, disc.dyn, disc.length, disc.time, disc.tempo)
    call("msq_midi_decode", ptr(rows), B, L, rows.stride(0), d, res_per_beat, out.pitch.shape[1], ptr(out.pitch),
         ptr(out.channel), ptr(out.dyn), ptr(out.tempo), ptr(out.beat_start), ptr(out.beat_end), ptr(out.t_start),
         ptr(out.t_end), ptr(out.count), stream())
    return out


def decode(token_seq, disc: Discretization = DEFAULT_DISC):
    """processing.decode(token_seq) drop-in: one row (tensor or list) -> list of MIDI_note."""
    t = torch.as_tensor(token_seq, dtype=torch.int64)
    if not t.is_cuda:
        t = t.cuda()
    return decode_batch(t.contiguous(), disc).notes(0)


def encode_batch(songs, disc: Discretization = DEFAULT_DISC, res_per_beat: int = BAR_RES, device="cuda"):
    """songs: list of lists of MIDI_note (sorted by time_start; times in
    seconds, integer tempos). Returns (tokens: list of int64 numpy arrays,
    beats: list of int64 [n, 2] arrays = the notes' adjusted time_start /
    time_end) from one msq_midi_encode launch."""
    import numpy as np
    off = np.zeros(len(songs) + 1, dtype=np.int64)
    off[1:] = np.cumsum([len(s) for s in songs])
    n = int(off[-1])
    cols = np.zeros((4, max(n, 1)), dtype=np.int32)
    times = np.zeros((2, max(n, 1)), dtype=np.float64)
    k = 0
    for song in songs:
        for m in song:
            cols[:, k] = (int(m.pitch), int(m.channel), int(m.dynamic), int(m.tempo))
            times[:, k] = (float(m.time_start), float(m.time_end))
            k += 1
    dev = torch.device(device)
    c = torch.from_numpy(cols).to(dev)
    t = torch.from_numpy(times).to(dev)
    o = torch.from_numpy(off).to(dev)
    tok = torch.empty(max(5 * n, 1), dtype=torch.int64, device=dev)
    beats = torch.empty(2, max(n, 1), dtype=torch.int64, device=dev)
    count = torch.empty(max(len(songs), 1), dtype=torch.int64, device=dev)
    d = (ctypes.c_int64 * 6)(disc.pitch, disc.channel, disc.dyn, disc.length, disc.time, disc.tempo)
    call("msq_midi_encode", ptr(c[0]), ptr(c[1]), ptr(c[2]), ptr(c[3]), ptr(t[0]), ptr(t[1]), ptr(o), len(songs), d,
         res_per_beat, ptr(tok), ptr(beats[0]), ptr(beats[1]), ptr(count), stream())
    tok, beats, count = tok.cpu().numpy(), beats.cpu().numpy(), count.cpu().numpy()
    out_t = [tok[5 * off[i]:5 * off[i] + count[i]].copy() for i in range(len(songs))]
    out_b = [beats[:, off[i]:off[i + 1]].T.copy() for i in range(len(songs))]
    return out_t, out_b


def encode(midi_notes, disc: Discretization = DEFAULT_DISC):
    """processing.encode(midi_notes) drop-in: returns the token list and, like
    the reference's adjust_note_time, rewrites each note's time_start /
    time_end to integer beats."""
    if not midi_notes:
        raise IndexError("list index out of range")  # adjust_note_time reads midi_notes[0]
    toks, beats = encode_batch([midi_notes], disc)
    for m, (bs, be) in zip(midi_notes, beats[0]):
        m.time_start, m.time_end = int(bs), int(be)
    return [int(x) for x in toks[0]]


def extract_midi(path):
    """processing.extract_midi (processing.py:57-83) over midiseq.smf: the
    non-drum notes of a .mid file with the tempo (round(bpm)) in force at each
    note's start, de-duplicated and sorted by start time."""
    from . import smf
    raw, tempos = smf.read_midi(path)
    notes = []
    for p, a, b, vel, prog, drum in raw:
        if drum:
            continue
        k = 0
        while k + 1 < len(tempos) and tempos[k + 1][0] <= a:
            k += 1
        notes.append(MIDI_note(pitch=abs(p), time_start=abs(a), time_end=abs(b), dynamic=abs(vel), channel=abs(prog),
                               tempo=round(tempos[k][1])))
    return sorted(list(set(notes)), key=lambda n: n.time_start)


def preprocess_midi_files(midi_folder, preprocess_folder, min_notes=200, batch=64):
    """processing.preprocess_midi_files (processing.py:24-55): every
    <midi_folder>/<model>/<band>/<song>.mid(i) with >= min_notes notes ->
    <preprocess_folder>/<model>/<band>/<song>.npy token row; existing outputs
    are kept. Songs are encoded ``batch`` at a time on the device."""
    import os
    from pathlib import Path
    import numpy as np
    todo = []
    for root, _, files in os.walk(midi_folder):
        for fn in files:
            if fn.lower().endswith((".mid", ".midi")):
                pth = Path(root) / fn
                model, band = pth.parts[-3], pth.parts[-2]
                dst = Path(preprocess_folder) / model / band / pth.stem
                if not os.path.exists(str(dst) + ".npy"):
                    todo.append((pth, dst))
    written = []
    for i in range(0, len(todo), batch):
        songs, dsts = [], []
        for src, dst in todo[i:i + batch]:
            try:
                notes = extract_midi(str(src))
            except Exception:  # the reference skips unreadable files (bare except)
                continue
            if len(notes) < min_notes:
                continue
            songs.append(notes)
            dsts.append(dst)
        if not songs:
            continue
        toks, _ = encode_batch(songs)
        for dst, t in zip(dsts, toks):
            os.makedirs(dst.parent, exist_ok=True)
            np.save(str(dst) + ".npy", t.astype(np.int64))
            written.append(str(dst) + ".npy")
    return written

"""Token -> note decode of generated rows on the device.

Drop-in for ``processing.decode(token_seq)`` (processing/processing.py:171-214,
with revert_note_time :154-169) as called by scripts/generate_midi_combined.py
:143-156 on each generated row. ``decode_batch`` runs ONE launch of
``msq_midi_decode`` (csrc/midi.hip) over all B rows while they are still in
HBM; ``decode`` returns the reference's list of ``MIDI_note`` for one row.

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

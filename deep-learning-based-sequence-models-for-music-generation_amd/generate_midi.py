"""Composer-conditioned generation to .mid files: the caller of the decode hot
path, mirroring scripts/generate_midi_combined.py:16-187.

Per band (composer) folder of the token store: B prompts = the first batch of
the band's sequential loader (random 2048-token windows of its shuffled songs,
metadata vector of the band; zeroed with no_metadata, :110-121), ``generate``
of ``length`` new tokens per model (:122-139), token -> note decode of every
row — the whole row with ``retain``, else its last length + 300 tokens
(:140-156) — in ONE device launch per model (midi.decode_batch), and one .mid
per row via midiseq.smf (:157-186), named generated_<band>_<model>_<i>.mid
under <output>/<model>[_no_meta|_removed_meta]/<band>/ (or <output>/combined/
<band>/ with combined_path). Bands whose last output exists, or with fewer
than two files, are skipped (:62-95).

Rows the reference's decode would reject (no complete note -> IndexError, a
zero tempo before the last note -> ZeroDivisionError) abort the reference
script; here they are reported and skipped."""
import os
import random

import torch

from . import midi, smf
from .config import BATCH_SIZE, BLOCK_LEN
from .data import DatasetLoader
from .generate import generate


def out_dirs(output_path, band, no_metadata=False, removed_metadata=False):
    """Output folder per model kind (generate_midi_combined.py:68-80)."""
    suffix = "_no_meta" if no_metadata else "_removed_meta" if removed_metadata else ""
    d = {k: os.path.join(output_path, f"{k}{suffix}", band) for k in ("mamba", "transformer")}
    d["combined"] = os.path.join(output_path, "combined", band)
    return d


def band_prompts(data_root, band, metadata, B, block_len=BLOCK_LEN, device="cuda", seed=None):
    """The first batch of the band's full loader (:111-119): src [A, T], meta [A, 6]."""
    loader = DatasetLoader(os.path.join(data_root, band), metadata, batch_size=B, block_len=block_len, device=device,
                           seed=seed)
    for src, _, meta in loader.get_dataloader_full():
        return src, meta
    raise ValueError(f"no songs for {band}")


def write_rows(seqs, names, out_dir, keep):
    """Decode the rows' last ``keep`` tokens (all with keep=None) in one launch
    and write one .mid per row; returns (written paths, skipped (name, reason))."""
    rows = seqs if keep is None else seqs[:, -keep:]
    nb = midi.decode_batch(rows.contiguous())
    written, skipped = [], []
    os.makedirs(out_dir, exist_ok=True)
    for i, name in enumerate(names):
        try:
            notes = nb.notes(i)
        except (IndexError, ZeroDivisionError) as e:
            skipped.append((name, f"{type(e).__name__}: {e}"))
            continue
        path = os.path.join(out_dir, name)
        smf.note_to_midi(notes, path)
        written.append(path)
    return written, skipped


def generate_band(models, band, data_root, metadata, output_path, length, B=BATCH_SIZE, retain=False,
                  no_metadata=False, removed_metadata=False, combined_path=False, block_len=BLOCK_LEN,
                  mode="exact", rng=None, device="cuda", seed=None):
    """One band of the reference's loop (:60-187). models: {"mamba": m,
    "transformer": m} (any subset). Returns the list of written .mid paths."""
    folder = os.path.join(data_root, band)
    n_files = sum(os.path.isfile(os.path.join(folder, f)) for f in os.listdir(folder))
    if n_files < 2:
        print(f"Skipping {band} (not enough files: {n_files})")
        return []
    dirs = out_dirs(output_path, band, no_metadata, removed_metadata)
    first = next(iter(models))
    last = os.path.join(dirs["combined"] if combined_path else dirs[first], f"generated_{band}_{first}_{B - 1}.mid")
    if os.path.exists(last):
        print(f"Skipping {band} (already has output)")
        return []
    print(f"Processing band: {band}")
    written, done = [], 0
    while done < B:
        # a fixed seed gives each pass its own loader draw (the reference builds a
        # fresh randomly shuffled loader per pass)
        src, meta = band_prompts(data_root, band, metadata, B, block_len, device,
                                 None if seed is None else seed + done)
        src, meta = src[:B - done], meta[:B - done]
        A = src.shape[0]
        if no_metadata:
            meta = torch.zeros_like(meta)
        for kind, model in models.items():
            seqs = generate(model, block_len, src, meta, num_tokens=length, device=device, rng=rng,
                            return_tensor=True, mode=mode if kind == "mamba" else "exact")
            names = [f"generated_{band}_{kind}_{done + i}.mid" for i in range(A)]
            w, skipped = write_rows(seqs, names, dirs["combined"] if combined_path else dirs[kind],
                                    None if retain else length + 300)
            for name, why in skipped:
                print(f"  {name}: not written ({why})")
            written += w
        done += A
    return written


def band_list(data_root, reverse=False, randomize=False, composers="", rng=None):
    """Band folders in the reference's order options (:35-41)."""
    bands = [d for d in os.listdir(data_root) if os.path.isdir(os.path.join(data_root, d))]
    if reverse:
        bands = sorted(bands, reverse=True)
    if randomize:  # the reference assigns random.shuffle's None here; the intent is a shuffle
        (rng or random).shuffle(bands)
    if composers:
        bands = [c.strip() for c in composers.split(",")]
    return bands

"""Command-line generation (scripts/generate_midi_combined.py:16-187 on the
MI355X path):

  python generate_midi.py --length 2000 --transformer True --data_root <root> \\
      --metadata metadata.json --output_path out/ [--transformer_ckpt t.pth]

Same flags as the reference (``type=bool`` flags: any non-empty value is
true, as there). Checkpoints are reference-format .pth state_dicts loaded
with weights_only=True (the reference's cc.config.models paths are
site-specific); without one the model is random-init. --mode cached runs the
Mamba recurrent decode (exact while prompt + new <= context)."""
import argparse
import os
import random
import sys

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import _pkgload  # noqa: E402
import torch  # noqa: E402

_pkgload.load()
from midiseq.config import BATCH_SIZE, BLOCK_LEN  # noqa: E402
from midiseq.generate_midi import band_list, generate_band  # noqa: E402
from midiseq.train_parallel import load_model, new_model  # noqa: E402


def main():
    ap = argparse.ArgumentParser(description="Generation")
    ap.add_argument("--length", type=int, help="Number of generated tokens")
    ap.add_argument("--mamba", type=bool, default=False)
    ap.add_argument("--transformer", type=bool, default=False)
    ap.add_argument("--retain", type=bool, default=False)
    ap.add_argument("--reverse", type=bool, default=False)
    ap.add_argument("--randomize", type=bool, default=False)
    ap.add_argument("--no_metadata", type=bool, default=False)
    ap.add_argument("--removed_metadata", type=bool, default=False)
    ap.add_argument("--data_root", type=str, required=True)
    ap.add_argument("--metadata", type=str, required=True, help="metadata.json (band -> genres, year)")
    ap.add_argument("--output_path", type=str, default="output")
    ap.add_argument("--combined_path", type=bool, default=False)
    ap.add_argument("--composers", type=str, default="")
    ap.add_argument("--mamba_ckpt", type=str, default=None)
    ap.add_argument("--transformer_ckpt", type=str, default=None)
    ap.add_argument("--batch_size", type=int, default=BATCH_SIZE)
    ap.add_argument("--block_len", type=int, default=BLOCK_LEN)
    ap.add_argument("--mode", choices=["exact", "cached"], default="exact")
    ap.add_argument("--seed", type=int, default=None)
    args = ap.parse_args()
    if args.length is None:
        ap.error("--length is required")
    rng = random.Random(args.seed) if args.seed is not None else None
    if args.seed is not None:
        # the device sampler draws from torch's generator (as torch.multinomial
        # does in the reference), so --seed seeds it too
        torch.manual_seed(args.seed)
    models = {}
    for kind in ("mamba", "transformer"):
        if getattr(args, kind):
            ckpt = getattr(args, f"{kind}_ckpt")
            kw = {} if kind == "mamba" else {"block_len": args.block_len}
            m = load_model(kind, ckpt, **kw) if ckpt else new_model(kind, **kw).to("cuda")
            if not ckpt:
                print(f"note: no --{kind}_ckpt, {kind} is random-init")
            models[kind] = m.eval()
    if not models:
        ap.error("choose --mamba and/or --transformer")
    for band in band_list(args.data_root, args.reverse, args.randomize, args.composers, rng):
        generate_band(models, band, args.data_root, args.metadata, args.output_path, args.length,
                      B=args.batch_size, retain=args.retain, no_metadata=args.no_metadata,
                      removed_metadata=args.removed_metadata, combined_path=args.combined_path,
                      block_len=args.block_len, mode=args.mode, rng=rng, seed=args.seed)


if __name__ == "__main__":
    main()

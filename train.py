"""Command-line training entry (the reference's train.py / train_parallel.py):

  python train.py --model transformer --data <root> --metadata metadata.json
  python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \\
      train.py --model transformer --data <root> --metadata metadata.json

<root>/<band>/<song>.npy token files are loaded once into HBM (midiseq.data);
without --data the loop runs on synthetic grammar-cycled batches. One process
per GPU, RCCL gradient buckets, fused Adam (midiseq.train_parallel)."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import torch  # noqa: E402,F401

import _pkgload  # noqa: E402

_pkgload.load()
from midiseq.config import BLOCK_LEN, LEARNING_RATE  # noqa: E402
from midiseq.train_parallel import load_model, new_model, setup_distributed, train  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="transformer", choices=["transformer", "mamba"])
    ap.add_argument("--data", default=None, help="<root>/<band>/<song>.npy token store")
    ap.add_argument("--metadata", default=None, help="metadata.json (band -> genres, year)")
    ap.add_argument("--batch-size", type=int, default=2)
    ap.add_argument("--block-len", type=int, default=BLOCK_LEN)
    ap.add_argument("--test-ratio", type=float, default=0.2)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--lr", type=float, default=LEARNING_RATE)
    ap.add_argument("--augmentation", action="store_true")
    ap.add_argument("--parallel", action="store_true", help="DistributedSampler shards instead of per-rank weighted")
    ap.add_argument("--resume", default=None, help="reference-format .pth to start from")
    ap.add_argument("--save", default=None, help="pretrained dir: <save>/<model>/loss_..._time_....pth")
    ap.add_argument("--save-every", type=int, default=0)
    ap.add_argument("--seed", type=int, default=0)
    args = ap.parse_args()

    rank, local, world = setup_distributed()
    dev = f"cuda:{local}"
    kw = {} if args.model == "mamba" else {"block_len": args.block_len}
    model = load_model(args.model, args.resume, device=dev, **kw) if args.resume else new_model(args.model, **kw)
    data = None
    if args.data:
        from midiseq.data import DatasetLoader
        if not args.metadata:
            ap.error("--data needs --metadata")
        dl = DatasetLoader(args.data, args.metadata, batch_size=args.batch_size, test_ratio=args.test_ratio,
                           block_len=args.block_len, device=dev, parallel=args.parallel, rank=rank, world=world,
                           seed=args.seed, augmentation=args.augmentation)
        data = dl.get_dataloaders()[0]
    train(model, args.model, data=data, steps=args.steps, lr=args.lr, save_dir=args.save,
          save_every=args.save_every or (args.steps if args.save else 0))


if __name__ == "__main__":
    main()

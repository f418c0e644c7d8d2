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
from midiseq.config import BLOCK_LEN, EPOCHS, EVAL_INTERVAL, LEARNING_RATE, SAVE_INTERVAL  # noqa: E402
from midiseq.train_parallel import load_model, new_model, setup_distributed, train  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="transformer", choices=["transformer", "mamba"])
    ap.add_argument("--data", default=None, help="<root>/<band>/<song>.npy token store")
    ap.add_argument("--metadata", default=None, help="metadata.json (band -> genres, year)")
    ap.add_argument("--batch-size", type=int, default=2)
    ap.add_argument("--block-len", type=int, default=BLOCK_LEN)
    ap.add_argument("--test-ratio", type=float, default=0.2)
    ap.add_argument("--epochs", type=int, default=EPOCHS)
    ap.add_argument("--max-steps", type=int, default=None, help="stop after this many optimizer steps")
    ap.add_argument("--steps-per-epoch", type=int, default=100, help="synthetic data only")
    ap.add_argument("--lr", type=float, default=LEARNING_RATE)
    ap.add_argument("--augmentation", action="store_true")
    ap.add_argument("--parallel", action="store_true", help="DistributedSampler shards instead of per-rank weighted")
    ap.add_argument("--resume", default=None, help="reference-format .pth to start from")
    ap.add_argument("--save", default=None, help="pretrained dir: <save>/<model>/loss_..._time_....pth")
    ap.add_argument("--save-interval", type=int, default=SAVE_INTERVAL, help="epochs between saves")
    ap.add_argument("--eval-interval", type=int, default=EVAL_INTERVAL, help="steps between loss logs")
    ap.add_argument("--log-file", default=None, help="JSON training log (rank 0)")
    ap.add_argument("--seed", type=int, default=0)
    args = ap.parse_args()

    torch.manual_seed(args.seed)  # dropout seeds of the train step come from torch's generator
    rank, local, world = setup_distributed()
    dev = f"cuda:{local}"
    kw = {} if args.model == "mamba" else {"block_len": args.block_len}
    model = load_model(args.model, args.resume, device=dev, **kw) if args.resume else new_model(args.model, **kw)
    data = test_data = None
    if args.data:
        from midiseq.data import DatasetLoader
        if not args.metadata:
            ap.error("--data needs --metadata")
        dl = DatasetLoader(args.data, args.metadata, batch_size=args.batch_size, test_ratio=args.test_ratio,
                           block_len=args.block_len, device=dev, parallel=args.parallel, rank=rank, world=world,
                           seed=args.seed, augmentation=args.augmentation)
        data, test_data = dl.get_dataloaders()
    train(model, args.model, data=data, test_data=test_data, epochs=args.epochs, max_steps=args.max_steps,
          eval_interval=args.eval_interval, save_interval=args.save_interval, lr=args.lr, save_dir=args.save,
          log_file=args.log_file, steps_per_epoch=args.steps_per_epoch)


if __name__ == "__main__":
    main()

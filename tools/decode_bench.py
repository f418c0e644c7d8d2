"""Mamba cached-decode leg of bench.py on its own (one JSON line), for
quick measurements and rocprofv3 kernel traces of the recurrent step.
Usage: python tools/decode_bench.py [B] [T0] [K]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import torch  # noqa: E402


def main():
    a = [int(x) for x in sys.argv[1:]]
    B, T0, K = (a + [64, 1024, 64][len(a):])[:3]
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    print(json.dumps(bench.mamba_decode_leg(dev, 0, 1, B=B, T0=T0, K=K)), flush=True)


if __name__ == "__main__":
    main()

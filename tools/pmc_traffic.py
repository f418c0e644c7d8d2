"""HBM traffic per kernel class from two rocprofv3 PMC passes over the same
bench command (MI355X_MICROARCH.md 'HBM': FETCH_SIZE and WRITE_SIZE in
separate passes, both in KB; on gfx950 FETCH_SIZE reports half the bytes of
wide coalesced reads, so it is doubled).

  rocprofv3 --pmc FETCH_SIZE -d <dir_f> -o run --output-format csv -- python bench.py ...
  rocprofv3 --pmc WRITE_SIZE -d <dir_w> -o run --output-format csv -- python bench.py ...
  python tools/pmc_traffic.py <dir_f> <dir_w> <train steps profiled> <out.json> [train|mamba]

Kernels map to bench.py's classes by name; bytes per class launch = bytes
per step / the class's launches per step (attention: 8 layers)."""
import csv
import glob
import json
import re
import sys
from collections import defaultdict

# (regex on the kernel name, class, class launches per train step)
CLASSES = [
    (r"flash_bwd_kv[345]|flash_bwd_dq|flash_bwd_pre|dqr_band_zero|flash_bwd_meta|gemm_bf16_kernel<1, 1, 5", "attn_bwd", 8),
    (r"flash_fwd3", "attn_fwd", 8),
    (r"attn_mask_kernel", "dropout_mask", 8),
    (r"colstats2|rowlse|cspart|cs_reduce|finish2|dbias_reduce|pad_table|wrange|mean_kernel", "loss", 1),
    (r"adam4?_kernel", "adam", 1),
    (r"ln_bwd|ln_reduce", "layernorm_bwd", 17),
    (r"gemm256_kernel<1, 1, 5|splitk_reduce", "gemm_dW", 33),
    # persistent 256 tile: forward and dX products (+ the ReLU-mask dX column-sum partials)
    (r"gemm256p_kernel|colsum_partials", "gemm_fwd_dX", 66),
    # FFN dX with the bias column sums (CS instantiation; bf16 template names come out mangled)
    (r"gemm256_kernel<0, 1|gemm256_kernelILi0ELi[01]ELi4E\w*Lb1E|colsum_partials", "gemm_dX", 8),
    # forward products and (with the transposed weight copies) the plain dX ones, + their split-K tails
    (r"gemm256_kernel<0, 0|gemm256_kernelILi0ELi0E|tail_epi_kernel|gemm_bf16_kernel<0, 0", "gemm_fwd", 58),
    # hipBLASLt kernels (the plain forward and dX products, both classes): bytes per step only
    (r"^Cijk_|^Custom_Cijk_", "gemm_blaslt", 1),
]


# Mamba train step (bench.py --only mamba: 10 Mamba2 layers, B=8, T=4096)
MAMBA_CLASSES = [
    (r"scan_fwd_kernel|ssd2::state_kernel|ssd2::pass_kernel|ssd2::out_kernel|state_kernel|pass_kernel|out_kernel", "ssd_fwd", 10),
    (r"scan_bwd_kernel|uterm_kernel|rpass_kernel|grad_kernel|dbc_reduce", "ssd_bwd", 10),
    (r"conv_fwd_kernel|conv_bwd_kernel", "mamba_conv", 20),
    (r"gnorm_fwd_kernel|gnorm_bwd_kernel|gnorm_bwd2_kernel", "mamba_gnorm", 20),
    (r"gemm256_kernel<1, 1, 5|splitk_reduce", "gemm_dW", 21),
    (r"gemm256p_kernel|gemm256_kernel<0|gemm256_kernelILi0E", "gemm_fwd_dX", 42),
    (r"colstats2|rowlse|cspart|cs_reduce|finish2|dbias_reduce|pad_table|wrange|mean_kernel", "loss", 1),
    (r"adam4?_kernel", "adam", 1),
]


def load(d, counter):
    files = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)
    rows = []
    for f in files:
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == counter:
                rows.append((r["Kernel_Name"], float(r["Counter_Value"])))
    return rows


def classify(name, classes=None):
    for pat, cls, n in classes or CLASSES:
        if re.search(pat, name):
            return cls, n
    return None, None


def main(dir_f, dir_w, steps, out, which="train"):
    steps = int(steps)
    classes = MAMBA_CLASSES if which == "mamba" else CLASSES
    tot = defaultdict(lambda: {"fetch_kb": 0.0, "write_kb": 0.0, "dispatches": 0})
    kern = defaultdict(lambda: {"fetch_kb": 0.0, "write_kb": 0.0, "n": 0})
    for counter, key, rows in (("FETCH_SIZE", "fetch_kb", load(dir_f, "FETCH_SIZE")),
                               ("WRITE_SIZE", "write_kb", load(dir_w, "WRITE_SIZE"))):
        for name, v in rows:
            short = re.sub(r"\(.*", "", name.replace("(anonymous namespace)::", "").replace("void ", ""))[:90]
            kern[short][key] += v
            if key == "fetch_kb":
                kern[short]["n"] += 1
            cls, _ = classify(name, classes)
            if cls is None:
                continue
            tot[cls][key] += v
            if key == "fetch_kb":
                tot[cls]["dispatches"] += 1
    res = {"source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of the bench step (tools/pmc_traffic.py)",
           "correction": "FETCH_SIZE x2 (gfx950 counts half of wide coalesced reads); KB x 1024 -> bytes",
           "train_steps_profiled": steps, "step": which, "classes": {}, "kernels": {}}
    for pat, cls, n in classes:
        if cls not in tot:
            continue
        t = tot[cls]
        per_step = (2 * t["fetch_kb"] + t["write_kb"]) * 1024 / steps
        res["classes"][cls] = {"hbm_bytes_per_step": per_step, "launches_per_step": n,
                               "hbm_bytes_per_launch": per_step / n,
                               "fetch_kb_per_step": t["fetch_kb"] / steps, "write_kb_per_step": t["write_kb"] / steps,
                               "dispatches_per_step": t["dispatches"] / steps}
    for k, t in sorted(kern.items(), key=lambda kv: -(2 * kv[1]["fetch_kb"] + kv[1]["write_kb"])):
        if t["n"] == 0:
            continue
        res["kernels"][k] = {"launches": t["n"], "read_mb_per_launch": round(2 * t["fetch_kb"] / 1024 / t["n"], 2),
                             "write_mb_per_launch": round(t["write_kb"] / 1024 / t["n"], 2)}
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:6])

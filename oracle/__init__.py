"""CPU ORACLE — test infrastructure only.

This package is a plain-PyTorch (CPU, fp32) and numpy restatement of the
reference's hot path (thorGabe123/Deep-Learning-Based-Sequence-Models-for-
Music-Generation @ 2025-08-24). It is the *checker*: only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
it. The product (``deep-learning-based-sequence-models-for-music-generation_amd``)
never imports it and has no CPU fallback.

Parity status: the Transformer, filtered-logit loss and sampler restatements
are PINNED against golden vectors produced by the reference's own code
(``tests/golden/make_golden.py`` loads the reference modules by file path in the
build container and records their outputs into ``tests/golden/*.npz``). The
Mamba2 restatement is pinned against HF ``transformers`` 5.15.0's pure-torch
Mamba2 mixer (the reference's ``mamba_ssm`` dependency is not vendored and its
version is unknown, so parity against ``mamba_ssm`` itself is *unpinned*).
"""

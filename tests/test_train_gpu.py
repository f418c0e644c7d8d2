"""The train() drop-in's epoch structure (train_parallel.py:169-235) on the
GPU: per epoch a pass over the train loader, model.eval() + validation loss
under no_grad over the test loader, a save every save_interval epochs named
by the average validation loss, and the final save."""
import json
from pathlib import Path

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_train_epochs_validation_and_saves(tmp_path):
    from midiseq import data
    from midiseq.train_parallel import evaluate, new_model, train
    rng = np.random.default_rng(3)
    arts = [{"name": "Mozart", "genres": ["classical"], "year_started": 1760},
            {"name": "Bach", "genres": ["baroque", "classical"], "year_started": 1700}]
    for b in ("Mozart", "Bach"):
        (tmp_path / "data" / b).mkdir(parents=True)
        for k in range(5):
            np.save(tmp_path / "data" / b / f"s{k}.npy", rng.integers(0, 17914, size=400).astype(np.int64))
    dl = data.DatasetLoader(str(tmp_path / "data"), {"artists": arts}, batch_size=2, test_ratio=0.2, block_len=128,
                            device="cuda", seed=0)
    tr, te = dl.get_dataloaders()
    model = new_model("transformer", n_embd=256, n_heads=2, n_layer=1, block_len=128).to("cuda")
    v0 = evaluate(model, te).item()
    assert model.training and np.isfinite(v0)
    log = train(model, "transformer", data=tr, test_data=te, epochs=2, eval_interval=2, save_interval=1,
                save_dir=str(tmp_path / "pre"), log_file=str(tmp_path / "log.json"))
    msgs = [e.get("message", "") for e in log]
    assert sum("Validation Loss" in m for m in msgs) == 2 and msgs[-1] == "Training complete!"
    saved = sorted((tmp_path / "pre" / "transformer").glob("loss_*_time_*.pth"))
    # epoch saves + the final one; the reference's name (2-decimal loss, time to
    # the second) makes saves with equal rounded loss in one second collide
    assert len(saved) >= 1
    sd = torch.load(saved[-1], map_location="cpu", weights_only=True)
    assert "blocks.0.sa.heads.1.query.weight" in sd
    assert json.loads(Path(tmp_path / "log.json").read_text())[0]["message"] == "Training started!"
    v1 = evaluate(model, te).item()
    assert np.isfinite(v1) and v1 != v0  # the optimizer moved the parameters

"""Host-side semantics of the training drop-in (train_parallel.py:49-65,
143-235): the model built by new_model carries the config's dropout, and the
epoch iterator follows the loader's length."""
from midiseq import config
from midiseq.train_parallel import SyntheticMIDI, _epoch_batches, new_model


def test_new_model_transformer_uses_config_dropout():
    m = new_model("transformer", n_layer=1, block_len=16)
    assert m.cfg.dropout == config.DROPOUT == 0.01
    assert m.training  # nn.Module default: dropout active in the training loop


def test_from_params_defaults_to_config_dropout():
    from types import SimpleNamespace
    from midiseq.transformer import TransformerConfig
    p = SimpleNamespace(n_embd=64, n_heads=4, n_layer=1, block_len=16, vocab_size=100, metadata_vocab_size=10)
    assert TransformerConfig.from_params(p).dropout == 0.01
    p.dropout = 0.2
    assert TransformerConfig.from_params(p).dropout == 0.2


def test_epoch_batches_follow_loader_length():
    class Loader:
        def __len__(self):
            return 3

        def __iter__(self):
            return iter([(i, i, i) for i in range(3)])
    assert len(list(_epoch_batches(Loader(), 100))) == 3
    syn = SyntheticMIDI(1, 8, "cpu", n_batches=2)
    assert len(list(_epoch_batches(syn, 5))) == 5


def test_config_values_match_reference_yaml():
    # configs/common/config.yaml:12-27
    assert (config.EPOCHS, config.EVAL_INTERVAL, config.SAVE_INTERVAL, config.LEARNING_RATE, config.TEST_RATIO,
            config.BATCH_SIZE, config.BLOCK_LEN) == (10000, 10, 10, 5e-5, 0.2, 2, 2048)

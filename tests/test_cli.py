"""Config C1 plumbing: FM on MovieLens-1M-shaped synthetic data through the
command line, on the CPU (the reference's own torch path), with CTR metrics."""
import numpy as np

from pytorchrec_amd import console_main
from pytorchrec_amd.metrics import AUC, LogLoss


def test_cli_fm_cpu_trains_and_evaluates():
    out = console_main.main(["--model_name", "fm", "--gpu", "-1", "--epoch", "2",
                             "--batch_size", "2048", "--train_rows", "20000", "--dev_rows", "4000",
                             "--lr", "0.1"])
    h = out["history"]
    assert len(h) == 2 and {"loss", "auc", "logloss"} <= set(h[0])
    assert all(np.isfinite(e["loss"]) for e in h)
    assert out["samples_per_s"] > 0


def test_metrics_match_definitions():
    rng = np.random.default_rng(0)
    z = rng.standard_normal(500)
    y = (rng.random(500) < 0.4).astype(float)
    # AUC = P(score_pos > score_neg) by brute force
    pos, neg = z[y > 0], z[y == 0]
    want = ((pos[:, None] > neg[None, :]).sum() + 0.5 * (pos[:, None] == neg[None, :]).sum()) / (
        len(pos) * len(neg))
    assert abs(AUC()(z, y) - want) < 1e-12
    p = 1 / (1 + np.exp(-z))
    want_ll = -np.mean(y * np.log(p) + (1 - y) * np.log(1 - p))
    assert abs(LogLoss()(z, y) - want_ll) < 1e-9
    assert AUC()(z, np.ones_like(z)) != AUC()(z, np.ones_like(z))  # nan: one class only


def test_cli_columnar_and_dataloader_paths_agree():
    """Both feeds run the CLI end to end (exact equality of the two feeds is
    checked in tests/test_loader.py with shuffling off; here fit shuffles, and
    the two feeds draw their permutations from different generators)."""
    outs = [console_main.main(["--model_name", "fm", "--gpu", "-1", "--epoch", "1",
                               "--batch_size", "1024", "--train_rows", "6000", "--dev_rows",
                               "2000", "--lr", "0.1", "--loader", ld])
            for ld in ("columnar", "dataloader")]
    assert [o["loader"] for o in outs] == ["columnar", "dataloader"]
    for o in outs:
        assert np.isfinite(o["history"][0]["loss"]) and 0.0 <= o["history"][0]["auc"] <= 1.0

"""The product's drop-in classes against the reference's own golden vectors, on
the CPU (no GPU needed): feature columns vs G8, FunkSVD initialisation /
checkpoint keys / both forward branches / one train step vs G3, G10, G11.
(The GPU runs of the same model are in test_gpu_pins.py.)"""
import numpy as np
import torch

from conftest import golden


def test_crossed_column_matches_reference_g8():
    from pytorchrec_amd.feature_column import CategoricalColumnWithIdentity, CrossedColumn
    g = golden("g8_columns.npz")
    cols = [CategoricalColumnWithIdentity(7, "a"), CategoricalColumnWithIdentity(5, "b"),
            CategoricalColumnWithIdentity(3, "c")]
    cross = CrossedColumn(cols)
    assert cross.category_num == int(g["category_num"])
    assert list(cross.coefficients) == list(g["coefficients"])
    batch = {k: torch.from_numpy(g[k]) for k in ("a", "b", "c")}
    got = cross.get_feature_data(batch)
    assert got.dtype == torch.int64
    assert np.array_equal(got.numpy(), g["crossed"])
    assert np.array_equal(cross.get_feature_ids(batch).numpy(), g["crossed"])


def test_numeric_column_matches_reference_g8_bit_exact():
    from pytorchrec_amd.feature_column import NormalizationMode, NumericColumn
    g = golden("g8_columns.npz")
    num = NumericColumn("x", min_value=-3.0, max_value=7.0, mean_value=2.0, std_value=2.9)
    batch = {"x": torch.from_numpy(g["x"])}
    for mode, key in ((NormalizationMode.NOP, "nop"), (NormalizationMode.MAX_MIN, "max_min"),
                      (NormalizationMode.Z_SCORE, "z_score")):
        got = num.get_feature_data(batch, mode).numpy()
        assert got.dtype == np.float32
        assert np.array_equal(got.view(np.uint32), g[key].view(np.uint32)), key


def _funk():
    from pytorchrec_amd.feature_column import CategoricalColumnWithIdentity
    from pytorchrec_amd.model import FunkSVD
    return FunkSVD(CategoricalColumnWithIdentity(50, "uid"), CategoricalColumnWithIdentity(37, "iid"),
                   CategoricalColumnWithIdentity(2, "label"), emb_size=8, random_seed=2020)


def test_funksvd_init_and_keys_match_reference():
    """Same seed -> bit-identical tables under the reference's state-dict keys."""
    g = golden("g10_funksvd_sgd_step.npz")
    sd = _funk().state_dict()
    assert set(sd) == {"u_embeddings.weight", "i_embeddings.weight"}
    assert np.array_equal(sd["u_embeddings.weight"].numpy().view(np.uint32),
                          g["u_before"].view(np.uint32))
    assert np.array_equal(sd["i_embeddings.weight"].numpy().view(np.uint32),
                          g["i_before"].view(np.uint32))


def test_funksvd_reference_checkpoint_round_trip(tmp_path):
    """A reference-keyed checkpoint loads (single-item forward == G3), saves back
    under the same keys, and a wrong shape is reported like torch does."""
    import pytest
    g = golden("g3_funksvd.npz")
    m = _funk()
    m.load_state_dict({"u_embeddings.weight": torch.from_numpy(g["u_table"]),
                       "i_embeddings.weight": torch.from_numpy(g["i_table"])})
    m.eval()
    with torch.no_grad():
        pred, tgt = m({"uid": torch.from_numpy(g["uid"]), "iid": torch.from_numpy(g["iid"]),
                       "label": torch.from_numpy(g["label"])})
    np.testing.assert_allclose(pred.numpy(), g["prediction"], rtol=1e-5, atol=1e-9)
    assert np.array_equal(tgt.numpy(), g["target"])
    path = tmp_path / "funk.pt"
    m.save_weights(str(path))
    sd = torch.load(path, weights_only=True)
    assert np.array_equal(sd["u_embeddings.weight"].numpy(), g["u_table"])
    m2 = _funk()
    m2.load_weights(str(path), torch.device("cpu"))
    assert torch.equal(m2.embeddings.weight, m.embeddings.weight)
    with pytest.raises(RuntimeError):
        m2.load_state_dict({"u_embeddings.weight": torch.zeros(49, 8),
                            "i_embeddings.weight": torch.zeros(37, 8)})
    with pytest.raises(RuntimeError):  # strict: a missing table key
        m2.load_state_dict({"u_embeddings.weight": torch.zeros(50, 8)})


def test_funksvd_sampled_branch_cpu_matches_reference_g11():
    g = golden("g11_funksvd_sampled.npz")
    m = _funk()
    m.load_state_dict({"u_embeddings.weight": torch.from_numpy(g["u_table"]),
                       "i_embeddings.weight": torch.from_numpy(g["i_table"])})
    m.eval()
    with torch.no_grad():
        pred, tgt = m({"uid": torch.from_numpy(g["uid"]), "iid": torch.from_numpy(g["iid"])})
    np.testing.assert_allclose(pred.numpy(), g["prediction"], rtol=1e-5, atol=1e-9)
    assert np.array_equal(tgt.numpy(), g["target"])


def test_funksvd_cpu_train_step_matches_reference_g10():
    g = golden("g10_funksvd_sgd_step.npz")
    m = _funk()
    m.compile(torch.optim.SGD(m.get_parameters(), lr=float(g["lr"])), torch.nn.MSELoss(), [],
              torch.device("cpu"))
    loss = float(m.train_step({"uid": torch.from_numpy(g["uid"]), "iid": torch.from_numpy(g["iid"]),
                               "label": torch.from_numpy(g["label"])})["loss"])
    np.testing.assert_allclose(loss, float(g["loss"]), rtol=1e-6)
    sd = m.state_dict()
    np.testing.assert_allclose(sd["u_embeddings.weight"].numpy(), g["u_after"], rtol=1e-5, atol=1e-8)
    np.testing.assert_allclose(sd["i_embeddings.weight"].numpy(), g["i_after"], rtol=1e-5, atol=1e-8)

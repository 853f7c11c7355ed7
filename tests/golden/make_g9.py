"""Generate golden fixture G9: the build's own CPU
restatement (oracle/restate.py) of the FM / DeepFM / DCN-v2 / DIN forwards in
fp64 AND fp32 on seeded synthetic inputs at B = 64, plus one full-size C2 case
(B = 4096, 26 tables x 38,462 rows, D = 16): an exact hash of its seeded inputs
and a checksum of its fp64 FM logits.

It pins the restatement against silent drift (tests/test_oracle_golden.py) and
hands the GPU tests (tests/test_gpu_g9.py) fixed expected outputs.  No reference
code is involved (the reference has no DeepFM / DCN-v2 / DIN).

    python tests/golden/make_g9.py
"""
from __future__ import annotations

import hashlib
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle import restate as R  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden", "g9_restatement.npz")

# small config: F fields of ROWS rows, D dims, ND dense, B samples
F, ROWS, D, ND, B = 8, 53, 8, 13, 64
MLP_U = (32, 16)
L_HIS, E = 20, 8
C2_F, C2_ROWS, C2_D, C2_ND, C2_B = 26, 38462, 16, 13, 4096


def small_inputs():
    rng = np.random.default_rng(909)
    d = F * D + ND
    a = {
        "tables": (rng.standard_normal((F, ROWS, D)) * 0.1).astype(np.float32),
        "wtabs": (rng.standard_normal((F, ROWS)) * 0.1).astype(np.float32),
        "ids": rng.integers(0, ROWS, (B, F)).astype(np.int64),
        "dense": rng.random((B, ND)).astype(np.float32),
        "dense_w": (rng.standard_normal(ND) * 0.1).astype(np.float32),
        "bias": np.float32(0.05),
        "label": (rng.random(B) < 0.25).astype(np.float32),
    }
    a["ids"][:4, 0] = [0, ROWS - 1, 0, ROWS - 1]  # edges + duplicates
    units = [d, *MLP_U]
    for i in range(len(MLP_U)):
        a[f"mlp_W{i}"] = (rng.standard_normal((units[i + 1], units[i])) / np.sqrt(units[i])).astype(np.float32)
        a[f"mlp_b{i}"] = (rng.standard_normal(units[i + 1]) * 0.05).astype(np.float32)
    a["out_W"] = (rng.standard_normal((1, MLP_U[-1])) / np.sqrt(MLP_U[-1])).astype(np.float32)
    a["out_b"] = np.array([0.02], np.float32)
    for i in range(3):
        a[f"cross_W{i}"] = (rng.standard_normal((d, d)) / np.sqrt(d)).astype(np.float32)
        a[f"cross_b{i}"] = (rng.standard_normal(d) * 0.05).astype(np.float32)
    a["din_q"] = (rng.standard_normal((B, E)) * 0.5).astype(np.float32)
    a["din_k"] = (rng.standard_normal((B, L_HIS, E)) * 0.5).astype(np.float32)
    lens = rng.integers(1, L_HIS + 1, B)
    a["din_valid"] = (np.arange(L_HIS)[None, :] < lens[:, None]).astype(np.uint8)
    a["din_att_W0"] = (rng.standard_normal((16, 4 * E)) / np.sqrt(4 * E)).astype(np.float32)
    a["din_att_b0"] = (rng.standard_normal(16) * 0.05).astype(np.float32)
    a["din_out_W"] = (rng.standard_normal((1, 16)) / 4.0).astype(np.float32)
    a["din_out_b"] = np.array([0.0], np.float32)
    return a


def small_outputs(a, dt):
    tabs, wt = list(a["tables"]), list(a["wtabs"])
    mlp = [(a[f"mlp_W{i}"], a[f"mlp_b{i}"]) for i in range(len(MLP_U))]
    out = (a["out_W"], a["out_b"])
    cross = [(a[f"cross_W{i}"], a[f"cross_b{i}"]) for i in range(3)]
    fm, _ = R.fm_logits(tabs, wt, a["ids"], a["dense"], a["dense_w"], a["bias"], dt)
    dfm = R.deepfm_logits(tabs, wt, a["ids"], a["dense"], a["dense_w"], a["bias"], mlp, out, dt)
    dcn = R.dcnv2_logits(tabs, a["ids"], a["dense"], cross, mlp, out, dt)
    u, s = R.din_pool(a["din_q"], a["din_k"], a["din_valid"], [(a["din_att_W0"], a["din_att_b0"])],
                      (a["din_out_W"], a["din_out_b"]), dt)
    return {"fm": fm, "deepfm": dfm, "deepfm_loss": R.bce_mean(dfm, a["label"], dt),
            "dcnv2": dcn, "din_u": u, "din_s": s}


def c2_inputs():
    """The full-size C2 case: tables and first-order column N(0, 0.1) (seed 4242),
    ids uniform (seed 0), dense U[0,1) (seed 2), dense weights (seed 5)."""
    rng = np.random.default_rng(4242)
    tables = (rng.standard_normal((C2_F, C2_ROWS, C2_D)) * 0.1).astype(np.float32)
    wtabs = (rng.standard_normal((C2_F, C2_ROWS)) * 0.1).astype(np.float32)
    ids = np.random.default_rng(0).integers(0, C2_ROWS, (C2_F, C2_B)).T.astype(np.int64)
    dense = np.random.default_rng(2).random((C2_B, C2_ND), dtype=np.float32)
    dense_w = (np.random.default_rng(5).standard_normal(C2_ND) * 0.1).astype(np.float32)
    return tables, wtabs, ids, dense, dense_w


def c2_hash(tables, wtabs, ids, dense, dense_w) -> str:
    h = hashlib.sha256()
    for x in (tables, wtabs, ids, dense, dense_w):
        h.update(np.ascontiguousarray(x).tobytes())
    return h.hexdigest()


def c2_checksum(z):
    """Size-independent summary of the B = 4096 logits: sum, sum of |z|, the
    first 32 values."""
    z = np.asarray(z, np.float64)
    return np.array([z.sum(), np.abs(z).sum()]), z[:32].copy()


def main():
    a = small_inputs()
    arrays = dict(a)
    for name, dt in (("f64", np.float64), ("f32", np.float32)):
        for k, v in small_outputs(a, dt).items():
            arrays[f"{k}_{name}"] = np.asarray(v)
    tables, wtabs, ids, dense, dense_w = c2_inputs()
    arrays["c2_sha256"] = np.array(c2_hash(tables, wtabs, ids, dense, dense_w))
    z, _ = R.fm_logits(list(tables), list(wtabs), ids, dense, dense_w, 0.0, np.float64)
    arrays["c2_fm_sums"], arrays["c2_fm_head"] = c2_checksum(z)
    arrays["numpy_version"] = np.array(np.__version__)
    np.savez_compressed(OUT, **arrays)
    print("wrote", OUT, sorted(arrays))


if __name__ == "__main__":
    main()

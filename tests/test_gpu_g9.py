"""The interaction kernel (mrec_interact_fwd) against golden G9 (the build's fp64
restatement, tests/golden/make_g9.py): the small FM case and the full-size C2
case (B = 4096, 26 x 38,462 rows, D = 16) through its checksum.  fp32 bank, so
the north-star bar applies directly: 1e-5 relative to the magnitude
|z| + 1/2 sum_d (sum_f |v|)^2 (SURVEY.md §7 hard part 3)."""
import os
import sys

import numpy as np
import pytest
import torch

from conftest import golden
from oracle import ref

pytestmark = pytest.mark.gpu


def _interact_fp32(gpu, tables, wtabs, ids, dense, dense_w, bias):
    from pytorchrec_amd import _mrec
    from pytorchrec_amd.embedding import EmbeddingBank, interact
    assert _mrec.available(), "libmrec.so must be built and loadable on the GPU box"
    F, rows, D = tables.shape
    bank = EmbeddingBank([rows] * F, D, with_first_order=True, dtype=torch.float32, device=gpu)
    with torch.no_grad():
        bank.weight.zero_()
        for f in range(F):
            o = bank.row_offset[f]
            bank.weight[o:o + rows, :D] = torch.from_numpy(tables[f]).to(gpu)
            bank.weight[o:o + rows, D] = torch.from_numpy(wtabs[f]).to(gpu)
    idt = [torch.from_numpy(ids[:, f].astype(np.int32)).to(gpu) for f in range(F)]
    logit = interact(bank, idt, torch.from_numpy(dense).to(gpu), torch.from_numpy(dense_w).to(gpu),
                     torch.tensor([bias], dtype=torch.float32, device=gpu), fm2=True,
                     first_order=True)
    return logit.detach().cpu().numpy().astype(np.float64)


def test_g9_fm_small_fp32_bank(gpu):
    g = golden("g9_restatement.npz")
    z = _interact_fp32(gpu, g["tables"], g["wtabs"], g["ids"], g["dense"], g["dense_w"],
                       float(g["bias"]))
    v = np.stack([g["tables"][f][g["ids"][:, f]] for f in range(g["tables"].shape[0])], 1)
    den = np.abs(g["fm_f64"]) + ref.fm2_magnitude(v)
    assert np.max(np.abs(z - g["fm_f64"]) / den) <= 1e-5


def test_g9_full_size_c2_checksum(gpu):
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
    import make_g9
    g = golden("g9_restatement.npz")
    tables, wtabs, ids, dense, dense_w = make_g9.c2_inputs()
    assert make_g9.c2_hash(tables, wtabs, ids, dense, dense_w) == str(g["c2_sha256"])
    z = _interact_fp32(gpu, tables, wtabs, ids, dense, dense_w, 0.0)
    sums, head = make_g9.c2_checksum(z)
    v = np.stack([tables[f][ids[:32, f]] for f in range(tables.shape[0])], 1)
    den = np.abs(g["c2_fm_head"]) + ref.fm2_magnitude(v)
    assert np.max(np.abs(head - g["c2_fm_head"]) / den) <= 1e-5
    # the sum of 4096 logits, each within 1e-5 of its magnitude
    vall = np.stack([tables[f][ids[:, f]] for f in range(tables.shape[0])], 1)
    mag = float((np.abs(z) + ref.fm2_magnitude(vall)).sum())
    assert abs(sums[0] - g["c2_fm_sums"][0]) <= 1e-5 * mag
    assert abs(sums[1] - g["c2_fm_sums"][1]) <= 1e-5 * mag

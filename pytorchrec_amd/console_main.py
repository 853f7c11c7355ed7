"""Command-line entry — the reference's ``console_main.py`` + ``Task`` flow
(console_main.py:9-19, torchrec/task/Task.py:34-76) for the CTR models, config C1:

    python -m pytorchrec_amd.console_main --model_name fm --gpu -1 --epoch 1

Same argument names and meaning as the reference Task (gpu: -1 = CPU, model_name,
random_seed, epoch, batch_size, optimizer, lr, l2, loss, metrics, num_workers,
dev_freq).  The reference's readers need private dataset paths (const.py:9-18) and
its console_main fails upstream, so the data here is the
MovieLens-1M-shaped synthetic set of SURVEY.md §8(d) C1: uid 1..6040,
iid 1..3706 (0 = PAD), gender 2, age 7, occupation 21, year bucket 18 and 18 genre
binaries = 24 categorical fields, labels Bernoulli(0.575).
"""
from __future__ import annotations

import argparse
import json
import sys
import time

import torch

ML1M_FIELDS = ([("uid", 6041), ("iid", 3707), ("gender", 2), ("age", 7), ("occupation", 21),
                ("year", 18)] + [(f"genre_{g}", 2) for g in range(18)])


def synthetic_ml1m(n: int, seed: int):
    g = torch.Generator().manual_seed(seed)
    data = {}
    for name, card in ML1M_FIELDS:
        lo = 1 if name in ("uid", "iid") else 0
        data[f"c_c_{name}"] = torch.randint(lo, card, (n,), generator=g, dtype=torch.int32)
    data["label"] = (torch.rand(n, generator=g) < 0.575).to(torch.int32)
    return data


class _Rows(torch.utils.data.Dataset):
    def __init__(self, cols):
        self.cols = cols
        self.n = len(next(iter(cols.values())))

    def __len__(self):
        return self.n

    def __getitem__(self, i):
        return {k: v[i] for k, v in self.cols.items()}


def parse(argv=None):
    p = argparse.ArgumentParser(description="pytorchrec_amd CTR task (reference Task arguments)")
    p.add_argument("--task_name", default="normal", choices=["normal"])
    p.add_argument("--debug", type=int, default=1)
    p.add_argument("--gpu", type=int, default=-1, help="GPU index, -1 = CPU")
    p.add_argument("--model_name", default="fm", choices=["fm", "deepfm"])
    p.add_argument("--random_seed", type=int, default=2020)
    p.add_argument("--metrics", default="auc,logloss")
    p.add_argument("--epoch", type=int, default=1)
    p.add_argument("--batch_size", type=int, default=4096)
    p.add_argument("--optimizer", default="sgd", choices=["sgd", "adam"])
    p.add_argument("--lr", type=float, default=0.05)
    p.add_argument("--l2", type=float, default=0.0)
    p.add_argument("--loss", default="bce", choices=["bce"])
    p.add_argument("--num_workers", type=int, default=0)
    p.add_argument("--loader", default="columnar", choices=["columnar", "dataloader"],
                   help="columnar: packed pinned batches (pytorchrec_amd/loader.py); "
                        "dataloader: the reference's per-sample DataLoader path")
    p.add_argument("--dev_freq", type=int, default=1)
    p.add_argument("--emb_size", type=int, default=16)
    p.add_argument("--train_rows", type=int, default=1_000_209, help="ML-1M has 1,000,209 ratings")
    p.add_argument("--dev_rows", type=int, default=100_000)
    return p.parse_args(argv)


def main(argv=None) -> dict:
    a = parse(argv)
    from pytorchrec_amd.feature_column import CategoricalColumnWithIdentity
    from pytorchrec_amd.loss import get_loss
    from pytorchrec_amd.metrics import get_metric
    from pytorchrec_amd.model.models import get_model_type
    from pytorchrec_amd.utils.global_utils import set_torch_seed

    set_torch_seed(a.random_seed)
    device = torch.device("cpu") if a.gpu < 0 else torch.device("cuda", a.gpu)
    sparse = [CategoricalColumnWithIdentity(card, f"c_c_{name}") for name, card in ML1M_FIELDS]
    label = CategoricalColumnWithIdentity(2, "label")
    cls = get_model_type(a.model_name)
    kw = dict(emb_size=a.emb_size, random_seed=a.random_seed)
    if a.model_name == "fm":
        model = cls(sparse, label, **kw)
    else:
        model = cls(sparse, None, label, **kw)
    params = model.get_parameters()
    opt = (torch.optim.SGD(params, lr=a.lr, weight_decay=a.l2) if a.optimizer == "sgd"
           else torch.optim.Adam(params, lr=a.lr, weight_decay=a.l2))
    metrics = [get_metric(m) for m in a.metrics.split(",") if m.strip()]
    model.compile(opt, get_loss(a.loss)(), metrics, device)
    from pytorchrec_amd.loader import ColumnarDataset
    wrap = ColumnarDataset if a.loader == "columnar" else _Rows
    train = wrap(synthetic_ml1m(a.train_rows, a.random_seed))
    dev = wrap(synthetic_ml1m(a.dev_rows, a.random_seed + 1))
    t0 = time.perf_counter()
    history = model.fit(train, a.batch_size, a.epoch, dev_dataset=dev, verbose=1,
                        workers=a.num_workers, dev_freq=a.dev_freq)
    secs = time.perf_counter() - t0
    out = {"model": a.model_name, "device": str(device), "epochs": a.epoch, "loader": a.loader,
           "train_rows": a.train_rows, "samples_per_s": round(a.epoch * a.train_rows / secs, 1),
           "history": history}
    print(json.dumps(out), flush=True)
    return out


if __name__ == "__main__":
    main(sys.argv[1:])

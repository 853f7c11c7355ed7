"""Model runtime base — mirror of ``torchrec.model.IModel``
(torchrec/model/IModel.py:34-321), the caller of the hot path.

Kept from the reference, same names / argument meaning / errors:
  * ``__init__(random_seed)``: seed -> ``_init_weights()`` -> ``_reset_weights()``
    (normal(0, 0.01) for every module whose type name contains "Linear" or
    "Embedding"; IModel.py:37-68) — so subclasses store their columns and
    hyper-parameters BEFORE calling ``super().__init__``;
  * ``get_parameters`` (bias params get weight_decay 0, IModel.py:83-92);
  * ``compile`` type checks raising ``ValueError`` (IModel.py:94-114);
  * ``train_step`` = to_device -> forward -> loss -> zero_grad -> backward -> step
    (IModel.py:116-125);
  * ``fit`` / ``evaluate`` / ``predict`` loops, ``save_weights`` / ``load_weights``,
    ``save_best_weights`` / ``load_best_weights``; ``RuntimeError`` before compile.

MI355X additions (documented deviations):
  * ``compile`` fuses the embedding update into the backward when the optimizer
    is plain SGD (no momentum / weight decay / nesterov on the bank's group):
    identical arithmetic to dense SGD, but no full-table gradient exists
    (SURVEY.md §7 hard part 5).  Any other optimizer gets the dense gradient.
  * ``predict`` calls ``predict_step`` (the reference calls a missing
    ``evaluate_step`` at IModel.py:300 and cannot run).
  * metrics may be any callables ``metric(prediction, target) -> float`` with a
    ``name``; the reference's ranking metrics are out of scope.
"""
from __future__ import annotations

import copy
import ctypes
import os
from abc import ABC, abstractmethod
from typing import Dict, List, Optional

import numpy as np
import torch
from torch.nn import Module
from torch.nn.modules.loss import _Loss  # noqa
from torch.optim.optimizer import Optimizer

from pytorchrec_amd.utils.argument import IWithArguments
from pytorchrec_amd.utils.data_structure import tensor_to_device
from pytorchrec_amd.utils.global_utils import set_torch_seed


class IModel(Module, IWithArguments, ABC):
    """Model interface: ``forward(data: Dict[str, Tensor]) -> (prediction, target)``."""

    def __init__(self, random_seed: int = 2020, **kwargs):  # noqa
        set_torch_seed(random_seed)
        super().__init__()
        self.stop_training = False
        self.best_state_dict = None
        self._weights_version = 0  # bumped by every train step / load (save_best_weights)
        self.history: Optional[list] = None
        self._is_compiled = False
        self.compiled_optimizers: Optional[Optimizer] = None
        self.compiled_loss: Optional[_Loss] = None
        self.compiled_metrics: Optional[list] = None
        self.compiled_device: Optional[torch.device] = None
        self._init_weights()
        self._reset_weights()

    @abstractmethod
    def _init_weights(self):
        pass

    @staticmethod
    def _reset_weights_fn(m):
        if "Linear" in str(type(m)):
            torch.nn.init.normal_(m.weight, mean=0.0, std=0.01)
            if m.bias is not None:
                torch.nn.init.normal_(m.bias, mean=0.0, std=0.01)
        elif "Embedding" in str(type(m)):
            with torch.no_grad():
                torch.nn.init.normal_(m.weight, mean=0.0, std=0.01)
                if hasattr(m, "zero_pad_"):  # an EmbeddingBank's row-pitch pad columns
                    m.zero_pad_()

    def _reset_weights(self):
        self.apply(self._reset_weights_fn)

    # -- checkpoints (IModel.py:73-81, 314-321) --------------------------------
    def load_weights(self, filepath: str, device: torch.device):
        """Restore a checkpoint written by ``save_weights``: a single-file state dict
        (the reference's format) or a row-sharded checkpoint (index file + per-rank
        shard files, checkpoint.py) -- into this model sharded at any world size or
        unsharded; every bank reads only its own rows."""
        from pytorchrec_amd import checkpoint
        state = torch.load(filepath, map_location="cpu", weights_only=True)
        checkpoint.load_into(self, state, os.path.abspath(filepath))
        self.to(device)
        self._weights_version += 1

    def save_weights(self, filepath: str):
        """The reference's ``torch.save(state_dict)``; a model with row-sharded banks
        writes the row-sharded checkpoint instead (collective: every rank calls it;
        checkpoint.save_sharded), which never assembles a bank anywhere."""
        from pytorchrec_amd import checkpoint
        if checkpoint.has_sharded_banks(self):
            checkpoint.save_sharded(self, filepath)
        else:
            # the reference pickles with HIGHEST_PROTOCOL (IModel.py:79-81); torch >= 2.6
            # loads with weights_only=True, whose unpickler rejects protocol >= 4 frames,
            # so the default protocol keeps the file loadable safely (here and by the
            # reference's own torch.load on a current torch)
            checkpoint.save_file(self.state_dict(), filepath)
        self._last_saved = (os.path.abspath(filepath), self._weights_version)

    # -- row-sharded checkpoints -------------------------
    def global_state_dict(self, dst: Optional[int] = None) -> Dict:
        """``state_dict()`` with every row-sharded bank replaced by the full bank in
        the unsharded layout (host memory, assembled chunk by chunk: the GPUs never
        hold more than their shard + one chunk), so the keys and shapes are exactly
        those of the same model built without sharding (and of the reference's
        per-field tables via ``EmbeddingBank.table``).  ``dst``: only that rank
        receives the banks (the others get None for them).  Collective over the
        shard group.  For banks larger than one host's memory use ``save_weights``."""
        from pytorchrec_amd.sharding import ShardedEmbeddingBank
        sd = self.state_dict()
        for name, m in self.named_modules():
            if isinstance(m, ShardedEmbeddingBank):
                sd[(name + "." if name else "") + "weight"] = m.gather_global(dst=dst)
        return sd

    def load_global_state_dict(self, state_dict: Dict, strict: bool = True):
        """Load a checkpoint in the unsharded layout (``global_state_dict`` or a
        single-GPU ``state_dict``); each row-sharded bank keeps its own rows."""
        from pytorchrec_amd import checkpoint
        checkpoint.load_into(self, state_dict, None, strict=strict)
        self._weights_version += 1
        return self

    def save_best_weights(self):
        """The reference deep-copies the state dict to host memory (IModel.py:314-317).
        ModelCheckpoint calls this right after ``save_weights`` (ModelCheckpoint.py:
        82-91): when nothing trained since that save, the files just written ARE the
        best state, kept as hard links under ``<file>.best`` (no copy; a later save
        replaces the live files' inodes, checkpoint.py) -- a row-sharded bank is never
        copied to any host.  Else a host copy of this rank's state (its own shard of
        a sharded bank, never the whole bank).  Every rank calls it."""
        from pytorchrec_amd import checkpoint
        saved = getattr(self, "_last_saved", None)
        if (saved is not None and saved[1] == self._weights_version
                and checkpoint.has_sharded_banks(self)):  # unsharded: the reference's copy
            snap = saved[0] + ".best"
            try:
                checkpoint.link_snapshot(self, saved[0], snap)
                self.best_state_dict = {"__mrec_best_file__": snap}
                return
            except OSError:  # no hard links here (or across devices): the host copy below
                pass
        self.best_state_dict = copy.deepcopy(tensor_to_device(self.state_dict(), torch.device("cpu")))

    def load_best_weights(self):
        assert self.best_state_dict is not None
        path = self.best_state_dict.get("__mrec_best_file__")
        if path is not None:
            self.load_weights(path, self.compiled_device)
            return
        self.load_state_dict(self.best_state_dict)
        self.to(self.compiled_device)
        self._weights_version += 1

    def get_parameters(self):
        weight_p, bias_p = [], []
        for name, p in filter(lambda x: x[1].requires_grad, self.named_parameters()):
            (bias_p if "bias" in name else weight_p).append(p)
        return [{"params": weight_p}, {"params": bias_p, "weight_decay": 0.0}]

    # -- compile ----------------------------------------------------------------
    def compile(self, optimizer: Optimizer, loss: _Loss, metrics: List, device: torch.device):
        if not isinstance(optimizer, Optimizer):
            raise ValueError(f"optimizer参数不合法: {optimizer}")
        if not isinstance(loss, _Loss):
            raise ValueError(f"loss参数不合法: {loss}")
        if not isinstance(metrics, list) or not all(callable(m) for m in metrics):
            raise ValueError(f"metrics参数不合法: {metrics}")
        if not isinstance(device, torch.device):
            raise ValueError(f"device参数不合法: {device}")
        self.compiled_optimizers = optimizer
        self.compiled_loss = loss
        self.compiled_metrics = metrics
        self.compiled_device = device
        self.to(device)
        self._configure_embedding_update(optimizer)
        self._configure_dense_update(optimizer)
        self._is_compiled = True

    def flush_embedding_optimizers(self):
        """Dense-compatible fused Adam: bring every table row to the current step
        (EmbeddingBank.flush_optimizer) before the tables are read as a whole --
        evaluation, prediction, checkpoints."""
        for bank in self.embedding_banks():
            bank.flush_optimizer()

    def state_dict(self, *args, **kwargs):
        self.flush_embedding_optimizers()
        return super().state_dict(*args, **kwargs)

    def embedding_banks(self):
        from pytorchrec_amd.embedding import EmbeddingBank
        return [m for m in self.modules() if isinstance(m, EmbeddingBank)]

    def _configure_embedding_update(self, optimizer: Optimizer):
        """Fuse the table update into the backward when it is exactly the compiled
        optimizer's: plain SGD, Adagrad, row-wise Adagrad, Adam / the reference
        AdamW (pytorchrec_amd.optim.fused_spec; Adam dense-compatible through
        catch-up steps and ``flush_optimizer``)."""
        from pytorchrec_amd.optim import fused_spec
        from pytorchrec_amd.sharding import ShardedEmbeddingBank

        def plain_sgd(g, sharded=False):
            return (isinstance(optimizer, torch.optim.SGD) and g.get("momentum", 0) == 0
                    and not g.get("nesterov", False) and not g.get("maximize", False)
                    and g.get("weight_decay", 0) == 0
                    and (not sharded or g.get("dampening", 0) == 0))

        for bank in self.embedding_banks():
            if isinstance(bank, ShardedEmbeddingBank):
                g0 = optimizer.param_groups[0]
                sgd = plain_sgd(g0, sharded=True)
                spec = None if sgd else fused_spec(optimizer, g0)
                if not sgd and spec is None:
                    raise NotImplementedError(
                        "row-sharded tables train with a fused update: torch.optim.SGD (no "
                        "momentum, weight_decay, dampening or nesterov), Adagrad (no lr_decay / "
                        "weight_decay), optim.RowWiseAdagrad, torch.optim.Adam (no amsgrad) "
                        "or optim.AdamW")
                if spec is None:
                    bank.use_fused_sgd(g0["lr"], g0)
                else:
                    kind = spec.pop("kind")
                    bank.use_fused_optimizer(kind, g0, grad_scale=1.0 / bank.world, **spec)
                continue
            if self._dp_active():
                # a replicated (unsharded) bank under data parallelism: its dense
                # gradient goes through the same all-reduce as the dense tower, so
                # the replicas cannot drift apart (a fused per-rank update would
                # apply each rank's own batch only)
                bank.use_dense_grad()
                continue
            group = None
            for g in optimizer.param_groups:
                if any(p is bank.weight for p in g["params"]):
                    group = g
            spec = (fused_spec(optimizer, group) if group is not None and bank.weight.is_cuda
                    else None)
            if group is not None and plain_sgd(group):
                bank.use_fused_sgd(group["lr"], group)
            elif spec is not None:
                kind = spec.pop("kind")
                bank.use_fused_optimizer(kind, group, **spec)
            elif group is not None or bank.update != "sgd":
                bank.use_dense_grad()

    def _configure_dense_update(self, optimizer: Optimizer):
        """Plain SGD on one process: every dense parameter is updated inside its own
        backward kernel (weight-gradient GEMM / column-sum epilogue), which also
        refreshes the bf16 weight images — no gradient tensors, no optimizer or
        conversion kernels.  Identical to torch.optim.SGD(lr) for these groups.
        Data-parallel training keeps the gradients (they must be all-reduced first)."""
        comm = getattr(self, "dp_comm", None)
        dp = comm is not None and (comm.world > 1 or comm.force)
        for p in self.parameters():
            for a in ("_mrec_sgd_group", "_mrec_dp_group", "_mrec_dp_grad"):
                if hasattr(p, a):
                    delattr(p, a)
        self._dp_flat = None
        if not isinstance(optimizer, torch.optim.SGD):
            return
        plain = []
        for g in optimizer.param_groups:
            if (g.get("momentum", 0) == 0 and g.get("weight_decay", 0) == 0
                    and not g.get("nesterov", False) and not g.get("maximize", False)
                    and g.get("dampening", 0) == 0):
                plain += [(p, g) for p in g["params"]]
        if not dp:
            for p, g in plain:
                p._mrec_sgd_group = g
            return
        # data parallel on the GPU: the backward kernels write the dense gradients
        # into ONE flat fp32 buffer (a view per parameter, 16-B aligned rows), the
        # step all-reduces it once and applies SGD to every parameter (and its bf16
        # GEMM images) in one mrec_sgd_multi launch
        dp_ids = {id(p) for p in self._dp_params()}
        banks = {id(b.weight) for b in self.embedding_banks()}  # dense-grad replicated tables
        plain = [(p, g) for p, g in plain
                 if id(p) in dp_ids and id(p) not in banks and p.is_cuda and p.dim() <= 2
                 and p.is_contiguous()]
        if not plain or len(plain) > 16:
            return
        layout, off = [], 0
        for p, g in plain:
            n, k = (1, p.numel()) if p.dim() < 2 else p.shape
            ld = (k + 7) // 8 * 8
            layout.append((p, g, n, k, ld, off))
            off += n * ld
        flat = torch.zeros(max(off, 1), dtype=torch.float32, device=plain[0][0].device)
        for p, g, n, k, ld, o in layout:
            view = flat[o:o + n * ld].view(n, ld)[:, :k]
            p._mrec_dp_grad = view if p.dim() == 2 else view.reshape(-1)
            p._mrec_dp_group = g
        self._dp_flat = (flat, layout)
        self._dp_sgd_table = None
        from pytorchrec_amd.sharding import ShardedEmbeddingBank
        for b in self.embedding_banks():  # the owner apply runs the dense SGD (ABI 28)
            if isinstance(b, ShardedEmbeddingBank) and os.environ.get("MREC_DP_INLINE_SGD", "1") == "1":
                b.dp_inline_sgd = self._dp_inline_sgd

    def _dp_flat_step(self):
        """All-reduce the flat gradient buffer (sum) and apply SGD with lr / world to
        every parameter that owns a view of it, plus its cached bf16 images."""
        from pytorchrec_amd import _mrec
        flat, _ = self._dp_flat
        self.dp_comm.allreduce_sum_(flat)
        jobs = self._dp_sgd_jobs()
        arr = (_mrec.SgdJob * len(jobs))(*jobs)
        _mrec.call("mrec_sgd_multi", len(jobs), arr, _mrec.stream_handle())

    def _dp_inline_sgd(self):
        """Called by a row-sharded bank's backward right before its owner apply, when
        every dense gradient of the step is in the flat buffer (the interaction is the
        model's first op, so its backward runs last): the flat all-reduce now, and the
        SGD as a table of tiles the owner's apply launch runs beside the embedding
        update (mrec_emb_bwd_apply_wire_sgd) instead of a mrec_sgd_multi launch of its
        own -- the same jobs, the same bits.  train_step then skips _dp_flat_step.
        -> (device table, workgroups), or None (no flat buffer)."""
        from pytorchrec_amd import _mrec
        from pytorchrec_amd import dense as dense_ops
        if getattr(self, "_dp_flat", None) is None:
            return None
        dense_ops.flush_pending()  # (any deferred reduction still writing the flat buffer)
        flat, _ = self._dp_flat
        self.dp_comm.allreduce_sum_(flat)
        jobs = self._dp_sgd_jobs()
        key = tuple((j.w, j.g, j.N, j.K, j.ldw, j.ldg, j.lr, j.img_row, j.ld_row, j.img_tr,
                     j.ld_tr, j.img_kind) for j in jobs)
        cached = getattr(self, "_dp_sgd_table", None)
        if cached is None or cached[2] != key:
            lib = _mrec.lib()
            nb = int(lib.mrec_sgd_table_bytes())
            host = (ctypes.c_uint8 * nb)()
            blocks = ctypes.c_int32(0)
            arr = (_mrec.SgdJob * len(jobs))(*jobs)
            _mrec.call("mrec_sgd_table_build", len(jobs), arr, ctypes.addressof(host), nb,
                       ctypes.byref(blocks))
            table = torch.frombuffer(bytearray(host), dtype=torch.uint8).to(flat.device)
            cached = (table, int(blocks.value), key)
            self._dp_sgd_table = cached
        self._dp_inline_done = True
        return cached[0], cached[1]

    def _dp_sgd_jobs(self):
        """The flat buffer's SGD jobs (lr / world), marking the images they re-emit."""
        from pytorchrec_amd import _mrec
        flat, layout = self._dp_flat
        comm = self.dp_comm
        from pytorchrec_amd.dense import cached_images, images_updated
        jobs = []
        for p, g, n, k, ld, o in layout:
            kind, imgs = None, None
            if p.dim() == 2:  # re-emit the images the kernels use (tower first)
                for kind in ("tower", "rowtr"):
                    imgs = cached_images(p, kind)
                    if imgs is not None:
                        break
            wr, wt = imgs if imgs is not None else (None, None)
            packed = kind == "tower" and imgs is not None
            jobs.append(_mrec.SgdJob(p.data_ptr(), flat.data_ptr() + 4 * o, n, k,
                                     p.stride(0) if p.dim() == 2 else k, ld,
                                     float(g["lr"]) / comm.world,
                                     _mrec.ptr(wr), 0 if packed or wr is None else wr.stride(0),
                                     _mrec.ptr(wt), 0 if packed or wt is None else wt.stride(0),
                                     _mrec.IMG_TOWER if packed else _mrec.IMG_ROW_TR))
            if imgs is not None:
                images_updated(p, kind)
        return jobs

    # -- data parallel (one process per GPU) ------------------------
    def distribute(self, comm):
        """Make this replica data-parallel over ``comm`` (a sharding.ShardComm):
        rank 0's dense parameters are broadcast now, and every train_step averages
        the dense gradients over the ranks (one flat all-reduce) before the
        optimizer step.  Row-sharded tables exchange rows themselves; unsharded
        tables are replicated and train through the dense-gradient all-reduce."""
        self.dp_comm = comm
        if self._is_compiled:
            self._configure_embedding_update(self.compiled_optimizers)
        with torch.no_grad():
            for p in self._dp_params():
                comm.broadcast_(p.data)
        if self._is_compiled:
            self._configure_dense_update(self.compiled_optimizers)
        return self

    def _dp_active(self) -> bool:
        comm = getattr(self, "dp_comm", None)
        return comm is not None and (comm.world > 1 or comm.force)

    def _dp_params(self):
        from pytorchrec_amd.sharding import ShardedEmbeddingBank
        sharded = {id(b.weight) for b in self.embedding_banks()
                   if isinstance(b, ShardedEmbeddingBank)}
        return [p for p in self.parameters() if p.requires_grad and id(p) not in sharded]

    def _allreduce_dense_grads(self):
        params = [p for p in self._dp_params() if p.grad is not None]
        if not params:
            return
        flat = torch.cat([p.grad.reshape(-1) for p in params])
        self.dp_comm.allreduce_mean_(flat)
        o = 0
        for p in params:
            n = p.grad.numel()
            p.grad.copy_(flat[o:o + n].view_as(p.grad))
            o += n

    # -- steps ------------------------------------------------------------------
    def train_step(self, data: Dict):
        self.train()
        self._weights_version += 1
        data = tensor_to_device(data, self.compiled_device)
        fused = self._fused_loss_fn()
        if fused is not None:
            # output layer + loss (+ their gradients) in one kernel; same math as
            # self(data) followed by compiled_loss (BCEWithLogits, mean)
            loss = fused(data)
            self.compiled_optimizers.zero_grad()
            from pytorchrec_amd.dense import grad_one
            loss.backward(grad_one(loss.device))
        else:
            prediction, target = self(data)
            loss = self.compiled_loss(prediction, target)
            self.compiled_optimizers.zero_grad()
            loss.backward()
        comm = getattr(self, "dp_comm", None)
        if comm is not None and (comm.world > 1 or comm.force):
            if getattr(self, "_dp_inline_done", False):
                self._dp_inline_done = False  # done in the owner's apply launch
            elif getattr(self, "_dp_flat", None) is not None:
                self._dp_flat_step()
            self._allreduce_dense_grads()  # parameters outside the flat buffer
        self.compiled_optimizers.step(closure=None)
        return {"loss": loss}

    def _fused_loss_fn(self):
        """A model may provide ``fused_bce_loss(data)`` (the CTR models do); it is
        used when the compiled loss is BCEWithLogitsLoss."""
        from pytorchrec_amd.loss import BCEWithLogitsLoss
        fn = getattr(self, "fused_bce_loss", None)
        if fn is None or not isinstance(self.compiled_loss, BCEWithLogitsLoss):
            return None
        return fn

    def test_step(self, data):
        self.eval()
        data = tensor_to_device(data, self.compiled_device)
        prediction, target = self(data)
        return prediction, target

    def predict_step(self, data):
        self.eval()
        data = tensor_to_device(data, self.compiled_device)
        prediction, _ = self(data)
        return prediction

    def _loader(self, dataset, batch_size, shuffle=False, workers=0, drop_last=False):
        """A ``ColumnarDataset`` is fed by the pipelined columnar loader (one packed
        H2D copy per batch, overlapped with the steps; pytorchrec_amd/loader.py);
        any other dataset by the reference's per-sample DataLoader."""
        from pytorchrec_amd.loader import ColumnarDataset, ColumnarLoader
        if isinstance(dataset, ColumnarDataset):
            key = (id(dataset), int(batch_size), bool(shuffle), bool(drop_last))
            cache = self.__dict__.setdefault("_columnar_loaders", {})
            ld = cache.get(key)
            if ld is None or ld.device != self.compiled_device:
                ld = ColumnarLoader(dataset, batch_size, self.compiled_device, shuffle=shuffle,
                                    drop_last=drop_last)
                cache[key] = ld
            return ld
        from torch.utils.data import DataLoader
        return DataLoader(dataset=dataset, batch_size=batch_size, shuffle=shuffle,
                          num_workers=workers, drop_last=drop_last)

    def fit(self, dataset, batch_size: int, epochs: int, dev_dataset=None, train_mode=None,
            verbose: int = 1, callbacks=None, shuffle: bool = True, workers: int = 0,
            drop_last: bool = False, dev_batch_size: Optional[int] = None, dev_freq: int = 1):
        """Epoch loop of IModel.py:127-209 without the (out-of-scope) callback
        framework: per-epoch logs are appended to ``self.history``."""
        self._assert_compile_was_called()
        self.stop_training = False
        self.history = []
        for epoch in range(epochs):
            if hasattr(dataset, "train_neg_sample") and train_mode is not None and \
                    str(getattr(train_mode, "value", train_mode)) == "pair_wise":
                dataset.train_neg_sample()
            logs = {}
            for data in self._loader(dataset, batch_size, shuffle, workers, drop_last):
                logs = self.train_step(data)
            epoch_logs = {k: float(v.detach() if torch.is_tensor(v) else v) for k, v in logs.items()}
            self.check_embedding_flags()
            if dev_dataset is not None and (epoch + 1) % dev_freq == 0:
                epoch_logs.update(self.evaluate(dev_dataset, dev_batch_size or batch_size,
                                                verbose=verbose, workers=workers))
            self.history.append(epoch_logs)
            if verbose:
                print(f"epoch {epoch + 1}/{epochs}: " +
                      ", ".join(f"{k}={v:.5f}" for k, v in epoch_logs.items()))
            if self.stop_training:
                break
        return self.history

    @torch.no_grad()
    def evaluate(self, dataset, batch_size: int, verbose: int = 1, callbacks=None, workers: int = 0):
        self._assert_compile_was_called()
        self.flush_embedding_optimizers()
        preds, targets = [], []
        for data in self._loader(dataset, batch_size, workers=workers):
            p, t = self.test_step(data)
            preds.append(p.detach().float().cpu().numpy())
            targets.append(t.detach().float().cpu().numpy())
        predictions = np.concatenate(preds) if preds else np.zeros(0)
        target = np.concatenate(targets) if targets else np.zeros(0)
        return {getattr(m, "name", type(m).__name__): float(m(predictions, target))
                for m in self.compiled_metrics}

    @torch.no_grad()
    def predict(self, dataset, batch_size: int, verbose: int = 0, callbacks=None, workers: int = 0):
        self.flush_embedding_optimizers()
        preds = [self.predict_step(d).detach().float().cpu().numpy()
                 for d in self._loader(dataset, batch_size, workers=workers)]
        return np.concatenate(preds) if preds else np.zeros(0)

    def check_embedding_flags(self):
        """Raise any sticky device-side error of the model's embedding banks (exchange
        overflow / out-of-range ids of a row-sharded bank, an unfinished huge-segment
        update of a large-batch backward).  One sync per bank."""
        for bank in self.embedding_banks():
            chk = getattr(bank, "check_flags", None)
            if chk is not None:
                chk()

    def _assert_compile_was_called(self):
        if not self._is_compiled:
            raise RuntimeError("训练/测试前必须编译模型")

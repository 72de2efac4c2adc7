"""``paddle.Model`` high-level API: prepare / fit / evaluate / predict / save / load."""
from __future__ import annotations

import numpy as np
import torch

from . import checkpoint as ckpt
from .io import DataLoader, Dataset


class Model:
    def __init__(self, network, inputs=None, labels=None):
        self.network = network
        self._optimizer = self._loss = None
        self._metrics = []

    def prepare(self, optimizer=None, loss=None, metrics=None, amp_configs=None):
        self._optimizer, self._loss = optimizer, loss
        self._metrics = metrics if isinstance(metrics, (list, tuple)) else ([metrics] if metrics else [])

    def _dev(self):
        p = next(self.network.parameters(), None)
        return p.device if p is not None else torch.device("cpu")

    def _split(self, batch):
        batch = list(batch) if isinstance(batch, (list, tuple)) else [batch]
        d = self._dev()
        batch = [b.to(d) if torch.is_tensor(b) else torch.as_tensor(np.asarray(b)).to(d) for b in batch]
        return batch[:-1] if len(batch) > 1 else batch, batch[-1:] if len(batch) > 1 else []

    def train_batch(self, inputs, labels=None):
        self.network.train()
        out = self.network(*inputs)
        loss = self._loss(out, *labels)
        loss.backward()
        self._optimizer.step()
        self._optimizer.clear_grad()
        for m in self._metrics:
            m.update(m.compute(out, *labels))
        return float(loss)

    @torch.no_grad()
    def eval_batch(self, inputs, labels=None):
        self.network.eval()
        out = self.network(*inputs)
        for m in self._metrics:
            m.update(m.compute(out, *labels))
        return float(self._loss(out, *labels)) if self._loss is not None and labels else None

    def _loader(self, data, batch_size, shuffle, drop_last=False, num_workers=0):
        if isinstance(data, Dataset):
            return DataLoader(data, batch_size=batch_size, shuffle=shuffle, drop_last=drop_last,
                              num_workers=num_workers)
        return data

    def fit(self, train_data=None, eval_data=None, batch_size=1, epochs=1, eval_freq=1, log_freq=10, save_dir=None,
            save_freq=1, verbose=2, drop_last=False, shuffle=True, num_workers=0, callbacks=None):
        loader = self._loader(train_data, batch_size, shuffle, drop_last, num_workers)
        hist = []
        for ep in range(epochs):
            for m in self._metrics:
                m.reset()
            losses = []
            for batch in loader:
                x, y = self._split(batch)
                losses.append(self.train_batch(x, y))
            rec = {"epoch": ep, "loss": float(np.mean(losses)) if losses else None}
            for m in self._metrics:
                rec[m.name()] = m.accumulate()
            if eval_data is not None and (ep + 1) % eval_freq == 0:
                rec["eval"] = self.evaluate(eval_data, batch_size, verbose=0)
            if save_dir and (ep + 1) % save_freq == 0:
                self.save(f"{save_dir}/{ep}")
            hist.append(rec)
            if verbose:
                print(rec)
        return hist

    def evaluate(self, eval_data, batch_size=1, log_freq=10, verbose=2, num_workers=0, callbacks=None):
        loader = self._loader(eval_data, batch_size, False, num_workers=num_workers)
        for m in self._metrics:
            m.reset()
        losses = []
        for batch in loader:
            x, y = self._split(batch)
            l = self.eval_batch(x, y)
            if l is not None:
                losses.append(l)
        res = {"loss": float(np.mean(losses)) if losses else None}
        for m in self._metrics:
            res[m.name()] = m.accumulate()
        return res

    @torch.no_grad()
    def predict(self, test_data, batch_size=1, num_workers=0, stack_outputs=False, verbose=1, callbacks=None):
        loader = self._loader(test_data, batch_size, False, num_workers=num_workers)
        self.network.eval()
        outs = []
        for batch in loader:
            x, _ = self._split(batch)
            outs.append(self.network(*x).cpu().numpy())
        return [np.concatenate(outs)] if stack_outputs else [outs]

    def save(self, path, training=True):
        ckpt.save(self.network.state_dict(), path + ".pdparams")
        if training and self._optimizer is not None:
            ckpt.save(self._optimizer.state_dict(), path + ".pdopt")

    def load(self, path, skip_mismatch=False, reset_optimizer=False):
        import os

        sd = ckpt.load(path + ".pdparams")
        self.network.set_state_dict(sd) if hasattr(self.network, "set_state_dict") else \
            self.network.load_state_dict(sd)
        if not reset_optimizer and self._optimizer is not None and os.path.exists(path + ".pdopt"):
            self._optimizer.set_state_dict(ckpt.load(path + ".pdopt"))

    def parameters(self):
        return list(self.network.parameters())

    def summary(self, input_size=None, dtype=None):
        n = sum(p.numel() for p in self.network.parameters())
        t = sum(p.numel() for p in self.network.parameters() if p.requires_grad)
        return {"total_params": n, "trainable_params": t}

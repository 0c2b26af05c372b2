"""Synthetic datasets (no network access: every benchmark and test uses generated data).

``TeacherClassification`` draws Gaussian inputs and labels them with a fixed random "teacher"
network, so the task is learnable, non-trivial, and reproducible from a seed.  The default shape is
MNIST's (784 features, 10 classes, 60k train rows), matching the reference's MNIST tutorial sweep
(``docs/src/user/pytorch.rst:131-136`` of the reference).
"""
from __future__ import annotations

import math

import torch


def pad_to(n: int, m: int = 64) -> int:
    return (n + m - 1) // m * m


class TeacherClassification:
    """x ~ N(0, I_d), y = argmax(teacher(x)); inputs stored padded to a multiple of 64 in bf16."""

    def __init__(self, n_train: int = 60032, n_val: int = 1024, in_features: int = 784,
                 num_classes: int = 10, teacher_hidden: int = 128, batch_size: int = 128,
                 seed: int = 0, device=None, temperature: float = 0.5):
        self.device = torch.device(device) if device is not None else torch.device("cpu")
        self.in_features = in_features
        self.num_classes = num_classes
        self.batch_size = batch_size
        self.k_pad = pad_to(in_features)
        n_train = max(batch_size, n_train // batch_size * batch_size)
        self.n_train = n_train
        self.n_val = n_val
        gen = torch.Generator(device="cpu")
        gen.manual_seed(seed)
        w1 = torch.randn(in_features, teacher_hidden, generator=gen) / math.sqrt(in_features)
        w2 = torch.randn(teacher_hidden, num_classes, generator=gen) / math.sqrt(teacher_hidden)
        self.train_x, self.train_y = self._draw(n_train, gen, w1, w2, temperature)
        self.val_x, self.val_y = self._draw(n_val, gen, w1, w2, temperature)

    def _draw(self, n, gen, w1, w2, temperature):
        xs, ys = [], []
        chunk = 8192
        for i in range(0, n, chunk):
            m = min(chunk, n - i)
            x = torch.randn(m, self.in_features, generator=gen)
            logits = torch.tanh(x @ w1 * 2.0) @ w2
            noise = -torch.log(-torch.log(torch.rand(m, self.num_classes, generator=gen)
                                          .clamp_(1e-12, 1 - 1e-12)))
            y = torch.argmax(logits / temperature + noise * 0.1, dim=1)
            xp = torch.zeros(m, self.k_pad)
            xp[:, :self.in_features] = x
            xs.append(xp.to(torch.bfloat16))
            ys.append(y.to(torch.int32))
        return (torch.cat(xs).to(self.device).contiguous(), torch.cat(ys).to(self.device).contiguous())

    @property
    def batches_per_epoch(self) -> int:
        return self.n_train // self.batch_size

    def batch(self, step: int):
        """Minibatch ``step`` (cycling through the epoch in order): contiguous views, no copy."""
        i = (step % self.batches_per_epoch) * self.batch_size
        return self.train_x[i:i + self.batch_size], self.train_y[i:i + self.batch_size]

    def validation(self):
        return self.val_x, self.val_y

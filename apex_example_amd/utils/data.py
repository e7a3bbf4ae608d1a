"""Synthetic data (there is no network for datasets).

* :class:`SyntheticMNIST` - an MNIST-shaped (1x28x28, 10 classes, 60,000
  samples) map-style dataset, generated deterministically per index.  Each
  class has its own fixed stroke template plus per-sample noise and jitter, so
  the reference ConvNet actually learns it (loss falls) - a stand-in for
  ``torchvision.datasets.MNIST`` with the same ``(image, label)`` contract
  (``ToTensor`` range [0, 1], float32) and usable with ``DistributedSampler``.
* :func:`image_batch` / :func:`token_batch` - on-device random batches for
  throughput benchmarks (generated once per rank, seeded by rank).
* :func:`str2bool` - a correct argparse bool (the reference's ``type=bool``
  makes ``--apex_enabled False`` truthy).
"""
from __future__ import annotations

import argparse

import torch


def str2bool(v):
    if isinstance(v, bool):
        return v
    s = str(v).strip().lower()
    if s in ("1", "true", "t", "yes", "y", "on"):
        return True
    if s in ("0", "false", "f", "no", "n", "off", ""):
        return False
    raise argparse.ArgumentTypeError("expected a boolean, got %r" % v)


class SyntheticMNIST(torch.utils.data.Dataset):
    def __init__(self, n=60000, num_classes=10, seed=0, noise=0.25):
        self.n = n
        self.num_classes = num_classes
        self.seed = seed
        self.noise = noise
        g = torch.Generator().manual_seed(seed)
        # class templates: a few random bright strokes on a 28x28 canvas
        t = torch.zeros(num_classes, 28, 28)
        for c in range(num_classes):
            for _ in range(4):
                r0, c0 = torch.randint(4, 20, (2,), generator=g).tolist()
                if torch.rand(1, generator=g).item() < 0.5:
                    t[c, r0:r0 + 2, c0:c0 + 8] = 1.0
                else:
                    t[c, r0:r0 + 8, c0:c0 + 2] = 1.0
        self.templates = t
        self.labels = torch.randint(0, num_classes, (n,), generator=g)

    def __len__(self):
        return self.n

    def __getitem__(self, i):
        label = int(self.labels[i])
        g = torch.Generator().manual_seed(self.seed * 1_000_003 + int(i))
        dr, dc = torch.randint(-2, 3, (2,), generator=g).tolist()
        img = torch.roll(self.templates[label], shifts=(dr, dc), dims=(0, 1))
        img = (img + self.noise * torch.rand(28, 28, generator=g)).clamp_(0, 1)
        return img.unsqueeze(0), label


def image_batch(batch, channels=3, size=224, num_classes=1000, device="cuda", seed=0,
                channels_last=True):
    g = torch.Generator(device="cpu").manual_seed(seed)
    x = torch.randn(batch, channels, size, size, generator=g).to(device)
    if channels_last:
        x = x.to(memory_format=torch.channels_last)
    y = torch.randint(0, num_classes, (batch,), generator=g).to(device)
    return x, y


def token_batch(batch, seq_len, vocab_size, device="cuda", seed=0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    return torch.randint(0, vocab_size, (batch, seq_len), generator=g).to(device)

"""CIFAR-10 without torchvision (the reference's DataloaderFactory.cifar10 path,
examples/__init__.py:557-652, reads torchvision.datasets.CIFAR10).

Reads the official binary release (``cifar-10-batches-bin/data_batch_{1..5}.bin`` and
``test_batch.bin``: records of 1 label byte + 3072 pixel bytes, CHW) or an ``.npz`` with
``x_train/y_train/x_test/y_test`` (uint8 NHWC or NCHW).  Nothing is downloaded and nothing is
unpickled.  Batches are assembled on the device: the training transform is the reference's
RandomCrop(32, padding=4) + RandomHorizontalFlip + Normalize(CIFAR mean/std), applied per sample
from a seeded generator; validation is Normalize only.  Under torch.distributed every rank reads
its own 1/world share of a per-epoch shuffled index (DistributedSampler semantics).
"""
from __future__ import annotations

import os

import numpy as np
import torch

MEAN = (0.4914, 0.4822, 0.4465)
STD = (0.2023, 0.1994, 0.2010)
RECORD = 1 + 3 * 32 * 32


def _read_bin(path):
    raw = np.fromfile(path, dtype=np.uint8)
    if raw.size % RECORD:
        raise ValueError(f"{path}: not a CIFAR-10 binary batch ({raw.size} bytes)")
    raw = raw.reshape(-1, RECORD)
    return raw[:, 1:].reshape(-1, 3, 32, 32), raw[:, 0].astype(np.int64)


def load_cifar10(root):
    """(x_train uint8 [N,3,32,32], y_train int64, x_test, y_test) from ``root``."""
    bindir = os.path.join(root, "cifar-10-batches-bin")
    if os.path.isdir(bindir) or os.path.isfile(os.path.join(root, "test_batch.bin")):
        d = bindir if os.path.isdir(bindir) else root
        tr = [_read_bin(os.path.join(d, f"data_batch_{i}.bin")) for i in range(1, 6)
              if os.path.isfile(os.path.join(d, f"data_batch_{i}.bin"))]
        if not tr:
            raise FileNotFoundError(f"no data_batch_*.bin under {d}")
        xte, yte = _read_bin(os.path.join(d, "test_batch.bin"))
        return np.concatenate([t[0] for t in tr]), np.concatenate([t[1] for t in tr]), xte, yte
    npz = root if root.endswith(".npz") else os.path.join(root, "cifar10.npz")
    if os.path.isfile(npz):
        with np.load(npz, allow_pickle=False) as z:
            out = []
            for k in ("x_train", "y_train", "x_test", "y_test"):
                v = z[k]
                if k.startswith("x") and v.shape[-1] == 3:
                    v = v.transpose(0, 3, 1, 2)
                out.append(np.ascontiguousarray(v.astype(np.uint8 if k.startswith("x") else np.int64)))
            return tuple(out)
    raise FileNotFoundError(f"no CIFAR-10 binary batches or cifar10.npz under {root} (nothing is downloaded)")


def write_cifar10_bin(path, x, y):
    """Write uint8 images [N,3,32,32] + labels as one CIFAR-10 binary batch (tests, tools)."""
    rec = np.empty((len(y), RECORD), np.uint8)
    rec[:, 0] = np.asarray(y, np.uint8)
    rec[:, 1:] = np.asarray(x, np.uint8).reshape(len(y), -1)
    rec.tofile(path)


class CifarLoader:
    """Iterates (images fp32 [B,3,32,32], labels int64 [B]) on ``device``."""

    def __init__(self, x, y, batch_size, device, train, seed=0, rank=0, world=1, drop_last=False):
        self.x = torch.from_numpy(np.ascontiguousarray(x)).to(device)
        self.y = torch.from_numpy(np.ascontiguousarray(y)).to(device)
        self.bs, self.dev, self.train = batch_size, device, train
        self.seed, self.rank, self.world, self.drop_last = seed, rank, world, drop_last
        self.epoch = 0
        self.mean = torch.tensor(MEAN, device=device).view(1, 3, 1, 1)
        self.std = torch.tensor(STD, device=device).view(1, 3, 1, 1)

    def set_epoch(self, epoch):
        self.epoch = epoch

    def _indices(self):
        n = self.y.numel()
        if self.train:
            g = torch.Generator().manual_seed(self.seed + self.epoch)
            idx = torch.randperm(n, generator=g)
        else:
            idx = torch.arange(n)
        if self.world > 1:  # DistributedSampler: pad to a multiple of world, then stride
            per = (n + self.world - 1) // self.world
            idx = torch.cat([idx, idx[: per * self.world - n]])[self.rank::self.world]
        return idx

    def __len__(self):
        n = len(self._indices())
        return n // self.bs if self.drop_last else (n + self.bs - 1) // self.bs

    def _augment(self, xb, g):
        """RandomCrop(32, padding=4) then RandomHorizontalFlip, per sample."""
        b = xb.shape[0]
        xp = torch.nn.functional.pad(xb, (4, 4, 4, 4))
        oy = torch.randint(0, 9, (b,), generator=g).to(self.dev)
        ox = torch.randint(0, 9, (b,), generator=g).to(self.dev)
        flip = (torch.rand(b, generator=g) < 0.5).to(self.dev)
        cols = ox[:, None] + torch.arange(32, device=self.dev)[None, :]
        cols = torch.where(flip[:, None], cols.flip(1), cols)
        return _rows(xp, oy).gather(3, cols[:, None, None, :].expand(b, 3, 32, 32))

    def __iter__(self):
        idx = self._indices().to(self.dev)
        g = torch.Generator().manual_seed(self.seed * 7919 + self.epoch * 31 + self.rank)
        for s in range(0, idx.numel(), self.bs):
            sel = idx[s:s + self.bs]
            if self.drop_last and sel.numel() < self.bs:
                break
            xb = self.x.index_select(0, sel).float().div_(255.0)
            if self.train:
                xb = self._augment(xb, g)
            yield (xb - self.mean) / self.std, self.y.index_select(0, sel)


def _rows(xp, oy):
    """rows oy .. oy+31 of each padded image [B,3,40,40] -> [B,3,32,40]"""
    b = xp.shape[0]
    ar = torch.arange(32, device=xp.device)
    r = (oy[:, None] + ar[None, :])[:, None, :, None].expand(b, 3, 32, xp.shape[3])
    return xp.gather(2, r)

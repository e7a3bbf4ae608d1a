"""Bit-exact mirror of the attention kernels' dropout hash (csrc/hip/attention.hip,
drop_base / drop_mix / drop_keep8) in int64 torch arithmetic, shared by the GPU parity
tests and the CPU statistics test."""
import torch

M32 = 0xFFFFFFFF
K_DROP_Q, K_DROP_K = 0x85EBCA77, 0xC2B2AE3D


def _mul32(a, c):
    return (a * c) & M32


def drop_base(seed, bh):
    x = (seed ^ _mul32(bh, 0x9E3779B1)) & M32
    x = x ^ (x >> 16)
    x = _mul32(x, 0x7FEB352D)
    x = x ^ (x >> 15)
    x = _mul32(x, 0x846CA68B)
    return x ^ (x >> 16)


def _umul24(x, c):
    return ((x & 0xFFFFFF) * (c & 0xFFFFFF)) & M32


def drop_mix(x):
    x = x ^ (x >> 16)
    x = _umul24(x, 0xE9846B) ^ (x >> 24)
    x = x ^ (x >> 13)
    x = _umul24(x, 0x8B3C2D) ^ (x >> 24)
    return x ^ (x >> 16)


def thr8(p):
    return 0 if p <= 0 else min(256, max(1, int(p * 256 + 0.5)))


def hash_bytes(B, H, S, seed, SK=None, device="cpu"):
    """[B, H, S(q), SK(k)] the byte of each (query, key) score's hash."""
    SK = S if SK is None else SK
    bh = torch.arange(B * H, dtype=torch.int64, device=device).view(B, H, 1, 1)
    q = torch.arange(S, dtype=torch.int64, device=device).view(1, 1, S, 1)
    key = torch.arange(SK, dtype=torch.int64, device=device).view(1, 1, 1, SK)
    x = (drop_base(seed, bh) + _mul32(q, K_DROP_Q) + _mul32(key >> 2, K_DROP_K)) & M32
    return (drop_mix(x) >> (8 * (key & 3))) & 0xFF


def keep_mask(B, H, S, seed, p, device="cpu"):
    """(keep mask [B, H, S, S], scale 1 / (1 - p_quantised))."""
    t = thr8(p)
    return hash_bytes(B, H, S, seed, device=device) >= t, (256.0 / (256 - t) if t < 256 else 0.0)

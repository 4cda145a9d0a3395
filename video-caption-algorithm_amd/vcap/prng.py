"""Portable counter-based PRNG for synthetic weights and frames.

SURVEY.md §8c asks for a seeded PRNG that does not depend on torch's RNG bit
stream, so the golden fixtures generated in the build container regenerate
bit-identically on the GPU box.  Every value is a pure function of
(seed, stream name, element index): splitmix64 over a 64-bit counter, then
24-bit uniforms (exact in fp32) and Box-Muller normals computed in float64.
"""
from __future__ import annotations

import zlib

import numpy as np

_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def _splitmix64(x: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = x + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def _stream_key(seed: int, name: str) -> np.uint64:
    h = zlib.crc32(name.encode("utf-8")) & 0xFFFFFFFF
    base = _splitmix64(np.array([(seed & 0xFFFFFFFF) << 32 | h], dtype=np.uint64))[0]
    return base


def _bits(seed: int, name: str, n: int, lane: int = 0) -> np.ndarray:
    key = _stream_key(seed, name)
    with np.errstate(over="ignore"):
        ctr = np.arange(n, dtype=np.uint64) * np.uint64(2) + np.uint64(lane)
        return _splitmix64(ctr ^ (key * np.uint64(0xD1342543DE82EF95)))


def uniform(seed: int, name: str, shape, low: float = 0.0, high: float = 1.0) -> np.ndarray:
    """U[low, high) as float32; 24-bit mantissa-exact base uniform."""
    n = int(np.prod(shape)) if len(shape) else 1
    u = (_bits(seed, name, n) >> np.uint64(40)).astype(np.float64) * (1.0 / 16777216.0)
    out = low + (high - low) * u
    return out.astype(np.float32).reshape(shape)


def normal(seed: int, name: str, shape, std: float = 1.0, mean: float = 0.0) -> np.ndarray:
    """N(mean, std^2) as float32 via Box-Muller on two independent 53-bit uniforms."""
    n = int(np.prod(shape)) if len(shape) else 1
    u1 = ((_bits(seed, name, n, 0) >> np.uint64(11)).astype(np.float64) + 1.0) * (1.0 / 9007199254740992.0)
    u2 = (_bits(seed, name, n, 1) >> np.uint64(11)).astype(np.float64) * (1.0 / 9007199254740992.0)
    z = np.sqrt(-2.0 * np.log(u1)) * np.cos(2.0 * np.pi * u2)
    return (mean + std * z).astype(np.float32).reshape(shape)


def imagenet_frames(seed: int, shape, name: str = "frames") -> np.ndarray:
    """Synthetic frames: pixel u~U[0,1) per (b,t,c,h,w), then ImageNet normalize.

    Mirrors core/preprocessing/frame_loader.py:34-40 (ToTensor -> Normalize with
    mean (0.485,0.456,0.406), std (0.229,0.224,0.225)); SURVEY.md §8d.
    """
    u = uniform(seed, name, shape)
    mean = np.array([0.485, 0.456, 0.406], dtype=np.float32).reshape((1,) * (len(shape) - 3) + (3, 1, 1))
    std = np.array([0.229, 0.224, 0.225], dtype=np.float32).reshape((1,) * (len(shape) - 3) + (3, 1, 1))
    return ((u - mean) / std).astype(np.float32)

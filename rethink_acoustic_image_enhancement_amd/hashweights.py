"""Deterministic, RNG-free synthetic weights and inputs (SURVEY.md §8c recipe).

Pretrained ``.pth`` files (``utils/download_weights.py:26-52`` in the reference) are not
reachable offline, so parity is anchored on weights that any machine regenerates bit-for-bit
from a state_dict key name and a flat element index:

    u(key, i) = splitmix64(fnv1a64(key) XOR i) mapped to [-1, 1)

* conv / linear weights: u / sqrt(fan_in)   (same support as torch's kaiming_uniform(a=sqrt 5))
* conv / linear biases:  u / sqrt(fan_in of the owning weight)
* LayerNorm weight: 1 + 0.1 u, LayerNorm bias: 0.1 u
* MDTA temperature: 1 + 0.5 u
* BatchNorm: gamma = 1 + 0.1 u, beta = 0.1 u, running_mean = 0.1 u, running_var = 1 + 0.5 |u|
* ``num_batches_tracked``: 0

Nothing here depends on torch's RNG, so the same tensors appear in this container (where the
golden fixtures are produced from the imported reference) and on the GPU box.
"""
from __future__ import annotations

import numpy as np

_M64 = (1 << 64) - 1


def fnv1a64(s: str) -> int:
    h = 0xCBF29CE484222325
    for b in s.encode("utf-8"):
        h ^= b
        h = (h * 0x100000001B3) & _M64
    return h


def _splitmix64(z: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = z + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return z


def hash_uniform(key: str, n: int) -> np.ndarray:
    """n float64 values in [-1, 1) for state_dict key ``key``."""
    idx = np.arange(n, dtype=np.uint64)
    z = _splitmix64(idx ^ np.uint64(fnv1a64(key)))
    return (z >> np.uint64(11)).astype(np.float64) * (2.0 / 9007199254740992.0) - 1.0


def _fan_in(shape) -> int:
    f = 1
    for s in shape[1:]:
        f *= int(s)
    return max(f, 1)


def hash_value(key: str, shape, weight_shapes: dict | None = None) -> np.ndarray:
    """Synthetic value for one state_dict entry (float32 array of ``shape``)."""
    shape = tuple(int(s) for s in shape)
    n = int(np.prod(shape)) if shape else 1
    leaf = key.rsplit(".", 1)[-1]
    u = hash_uniform(key, n)
    if leaf == "num_batches_tracked":
        return np.zeros(shape, dtype=np.int64)
    if leaf == "temperature":
        v = 1.0 + 0.5 * u
    elif leaf == "running_mean":
        v = 0.1 * u
    elif leaf == "running_var":
        v = 1.0 + 0.5 * np.abs(u)
    elif _is_norm_key(key, shape):
        v = (1.0 + 0.1 * u) if leaf == "weight" else 0.1 * u
    elif leaf == "weight":
        fan = _fan_in(shape)
        # ConvTranspose weights are [Cin, Cout, k...]: fan_in is Cout * prod(k)
        v = u / np.sqrt(fan)
    elif leaf == "bias":
        wkey = key[: -len("bias")] + "weight"
        wshape = (weight_shapes or {}).get(wkey)
        fan = _fan_in(wshape) if wshape is not None else max(n, 1)
        v = u / np.sqrt(fan)
    else:
        v = 0.1 * u
    return v.astype(np.float32).reshape(shape)


def _is_norm_key(key: str, shape) -> bool:
    # LayerNorm bodies (…norm1.body.weight) and BatchNorm affine params are 1-D scale vectors.
    if len(shape) != 1:
        return False
    return (".body." in key and ("norm1" in key or "norm2" in key)) or _is_bn_key(key)


def _is_bn_key(key: str) -> bool:
    # ASDQE DoubleConv: double_conv.{1,4}.* are BatchNorm2d (ASDQE/ASDQE_model.py:24-31)
    parts = key.split(".")
    return "double_conv" in parts and len(parts) >= 2 and parts[-2] in ("1", "4")


def hash_state_dict(shapes: dict) -> dict:
    """{key: shape} -> {key: float32/int64 numpy array} following the recipe above."""
    wshapes = {k: tuple(v) for k, v in shapes.items() if k.endswith("weight")}
    return {k: hash_value(k, s, wshapes) for k, s in shapes.items()}


def hash_images(key: str, shape, lo: float = 0.0, hi: float = 1.0) -> np.ndarray:
    """U[lo, hi) image batch from the same hash stream (inputs of SURVEY.md §8d configs)."""
    n = int(np.prod(shape))
    u = hash_uniform(key, n)
    return (lo + (hi - lo) * (u + 1.0) * 0.5).astype(np.float32).reshape(shape)


def hash_normal(key: str, shape) -> np.ndarray:
    """Box-Muller normal samples from two hash streams (ASDQE gt noise)."""
    n = int(np.prod(shape))
    u1 = (hash_uniform(key + "#bm1", n) + 1.0) * 0.5
    u2 = (hash_uniform(key + "#bm2", n) + 1.0) * 0.5
    u1 = np.maximum(u1, 1e-300)
    z = np.sqrt(-2.0 * np.log(u1)) * np.cos(2.0 * np.pi * u2)
    return z.astype(np.float32).reshape(shape)


def load_hash_weights(module) -> None:
    """Fill an nn.Module's state_dict in place with the hash recipe (torch imported lazily)."""
    import torch

    sd = module.state_dict()
    vals = hash_state_dict({k: tuple(v.shape) for k, v in sd.items()})
    new = {k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in vals.items()}
    module.load_state_dict(new, strict=True)

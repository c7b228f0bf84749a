"""Checkpoint ingest: the reference's on-disk layouts, loaded safely.

* BasicSR ``save_network`` writes ``{'params': sd}`` (optionally also ``'params_ema'``) with the
  ``module.`` prefix stripped (Train/basicsr/models/base_model.py:213-244); ``load_network``
  takes ``param_key`` with a fallback and strips ``module.`` (:246-309).
* The notebooks load ``torch.load(p)['params']`` strictly (KDLAE/KDLAE_T.ipynb:1074-1075).
* ASDQE saves a raw state_dict and loads it with ``strict=False`` (ASDQE/ASDQE_test.py:79).
* Restormer pretrained weights are a strict subset of KDLAE-T's keys (KDLAET.yml:83
  ``strict_load_g: false``).

Files are read with ``torch.load(..., weights_only=True)`` only; nothing in a checkpoint executes.
After loading, the module's parameters are the source of truth and the HIP handle repacks them on
the next forward.
"""
from __future__ import annotations

import torch


def read_state_dict(path: str, param_key: str = "params") -> dict:
    """The state_dict stored at ``path``: ``[param_key]`` if present, else ``params`` / ``params_ema``,
    else the file itself when it is already a flat state_dict; ``module.`` prefixes removed."""
    obj = torch.load(path, map_location="cpu", weights_only=True)
    sd = obj
    if isinstance(obj, dict):
        for k in (param_key, "params", "params_ema"):
            if k and k in obj and isinstance(obj[k], dict):
                sd = obj[k]
                break
    if not isinstance(sd, dict) or not all(torch.is_tensor(v) for v in sd.values()):
        raise RuntimeError(f"{path}: no state_dict found (keys {list(obj)[:8] if isinstance(obj, dict) else type(obj)})")
    return {(k[len("module."):] if k.startswith("module.") else k): v for k, v in sd.items()}


def load_checkpoint(model: torch.nn.Module, path: str, param_key: str = "params", strict: bool = True):
    """``model.load_state_dict`` from a reference checkpoint; returns (missing, unexpected) keys."""
    res = model.load_state_dict(read_state_dict(path, param_key), strict=strict)
    return list(res.missing_keys), list(res.unexpected_keys)

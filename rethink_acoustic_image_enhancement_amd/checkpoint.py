"""Checkpoint ingest: the reference's on-disk layouts, loaded safely.

* BasicSR ``save_network`` writes ``{'params': sd}`` (optionally also ``'params_ema'``) with the
  ``module.`` prefix stripped (Train/basicsr/models/base_model.py:213-244); ``load_network``
  takes ``param_key``, falls back to ``'params'`` when that key is absent, strips ``module.`` and,
  when not strict, drops keys whose shape differs from the module's (:246-309).
* The notebooks load ``torch.load(p)['params']`` strictly (KDLAE/KDLAE_T.ipynb:1074-1075,
  KDLAE/KDLAE-S.ipynb:109-110).
* ASDQE saves a raw state_dict (Train/ASDQE.py:210,215,219) and loads it with ``strict=False``
  (ASDQE/ASDQE_test.py:75-84).
* Restormer pretrained weights are a strict subset of KDLAE-T's keys (KDLAET.yml:82-83
  ``strict_load_g: false``).

Files are read with ``torch.load(..., weights_only=True)`` only; nothing in a checkpoint executes.
After loading, the module's parameters are the source of truth and the HIP handle repacks them on
the next forward.  The layouts are pinned by reference-written files in ``tests/golden/ckpt_*``.
"""
from __future__ import annotations

import torch


def _strip_module(sd: dict) -> dict:
    return {(k[len("module."):] if k.startswith("module.") else k): v for k, v in sd.items()}


def read_state_dict(path: str, param_key: str | None = "params") -> dict:
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
    return _strip_module(sd)


def load_checkpoint(model: torch.nn.Module, path: str, param_key: str = "params", strict: bool = True):
    """``model.load_state_dict`` from a reference checkpoint; returns (missing, unexpected) keys."""
    res = model.load_state_dict(read_state_dict(path, param_key), strict=strict)
    return list(res.missing_keys), list(res.unexpected_keys)


def load_network(net: torch.nn.Module, load_path: str, strict: bool = True, param_key: str | None = "params"):
    """BaseModel.load_network (Train/basicsr/models/base_model.py:281-309) for a bare module:
    ``param_key`` falls back to ``'params'`` only when it is absent and ``'params'`` exists (a
    missing key otherwise raises KeyError, as the reference does); ``param_key=None`` takes the
    file itself; ``module.`` is stripped; with ``strict=False`` a key whose shape differs from the
    module's is renamed ``<key>.ignore`` and so left out (:271-279).  Returns (missing, unexpected)."""
    load_net = torch.load(load_path, map_location="cpu", weights_only=True)
    if param_key is not None:
        if param_key not in load_net and "params" in load_net:
            param_key = "params"
        load_net = load_net[param_key]
    load_net = _strip_module(dict(load_net))
    if not strict:
        crt = net.state_dict()
        for k in list(load_net):
            if k in crt and crt[k].size() != load_net[k].size():
                load_net[k + ".ignore"] = load_net.pop(k)
    res = net.load_state_dict(load_net, strict=strict)
    return list(res.missing_keys), list(res.unexpected_keys)

"""Cache of derived weight layouts (concatenated / paired / pre-scaled copies of parameters).

The fused kernels want some weights in a different layout than nn.Linear stores them
(e.g. [x_proj; dt_proj] as one GEMM, gate/global rows interleaved for the fused gating
epilogue).  Those copies are built once per parameter version on the parameters' device
and rebuilt automatically when a parameter is modified, moved or reloaded.
"""

from __future__ import annotations

from typing import Callable, Iterable

import torch


def cached(module: torch.nn.Module, name: str, deps: Iterable[torch.Tensor], build: Callable[[], object]):
    sig = tuple((t.data_ptr(), t._version, str(t.device), tuple(t.shape)) for t in deps)
    store = module.__dict__.setdefault("_vasr_prepared", {})
    ent = store.get(name)
    if ent is None or ent[0] != sig:
        with torch.no_grad():
            ent = (sig, build())
        store[name] = ent
    return ent[1]

"""Import the reference's Python hot path on CPU (fixture generation ONLY).

Runs only in the build container, where ``/root/reference`` is mounted; nothing
on the GPU box imports this module.  The shim:

1. ``sys.path`` gets ``/root/reference`` so ``reconstruct`` / ``deep_sdf`` resolve
   to the reference's own sources (imported under fresh module names, never
   copied);
2. ``Tensor.cuda`` and ``torch.cuda.synchronize`` become no-ops (no GPU here);
3. ``addict``, ``plyfile`` and ``skimage.measure`` — imported at module level by
   ``reconstruct/utils.py:21-24`` but unused on the hot path — are stubbed.
   ``addict.Dict`` gets the attribute-dict behaviour ``ForceKeyErrorDict``
   (utils.py:82-84) relies on.

Bytecode writing is disabled so nothing is written into the read-only tree.
"""
from __future__ import annotations

import os
import sys
import types

REF = os.environ.get("DSR_REFERENCE", "/root/reference")


def available() -> bool:
    return os.path.isfile(os.path.join(REF, "reconstruct", "optimizer.py"))


class _AttrDict(dict):
    """Minimal addict.Dict: attribute access + recursive conversion of nested dicts."""

    def __init__(self, *args, **kwargs):
        super().__init__()
        for k, v in dict(*args, **kwargs).items():
            self[k] = self._conv(v)

    @classmethod
    def _conv(cls, v):
        if isinstance(v, dict) and not isinstance(v, _AttrDict):
            return cls(v)
        return v

    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError:
            return self.__missing__(k)

    def __missing__(self, k):
        raise KeyError(k)

    def __setattr__(self, k, v):
        self[k] = self._conv(v)


_loaded = None


def load():
    """Return a namespace with the reference modules (optimizer, loss, loss_utils, decoder, utils)."""
    global _loaded
    if _loaded is not None:
        return _loaded
    if not available():
        raise RuntimeError("reference tree not mounted at %s" % REF)
    sys.dont_write_bytecode = True
    import torch

    torch.Tensor.cuda = lambda self, *a, **k: self
    torch.cuda.synchronize = lambda *a, **k: None
    addict = types.ModuleType("addict")
    addict.Dict = _AttrDict
    sys.modules.setdefault("addict", addict)
    sys.modules.setdefault("plyfile", types.ModuleType("plyfile"))
    sk = types.ModuleType("skimage")
    skm = types.ModuleType("skimage.measure")
    sk.measure = skm
    sys.modules.setdefault("skimage", sk)
    sys.modules.setdefault("skimage.measure", skm)
    # the build's own package is also called ``reconstruct``: make sure the
    # reference's resolves here and restore the previous modules afterwards.
    saved = {k: sys.modules.pop(k) for k in list(sys.modules)
             if k == "reconstruct" or k.startswith("reconstruct.")
             or k == "deep_sdf" or k.startswith("deep_sdf.")}
    sys.path.insert(0, REF)
    try:
        import reconstruct.optimizer as optimizer
        import reconstruct.loss as loss
        import reconstruct.loss_utils as loss_utils
        import reconstruct.utils as utils
        import deep_sdf.deep_sdf_decoder as decoder
    finally:
        sys.path.remove(REF)
        ref_mods = {k: sys.modules.pop(k) for k in list(sys.modules)
                    if k == "reconstruct" or k.startswith("reconstruct.")
                    or k == "deep_sdf" or k.startswith("deep_sdf.")}
        sys.modules.update(saved)
    _loaded = types.SimpleNamespace(optimizer=optimizer, loss=loss, loss_utils=loss_utils,
                                    utils=utils, decoder=decoder, modules=ref_mods,
                                    AttrDict=_AttrDict)
    return _loaded


def build_decoder(state, specs):
    """Reference ``Decoder`` (deep_sdf_decoder.py:10-72) loaded with ``state`` (eval mode)."""
    import numpy as np
    import torch

    ref = load()
    dec = ref.decoder.Decoder(specs["CodeLength"], **specs["NetworkSpecs"])
    sd = {k[len("module."):]: torch.from_numpy(np.ascontiguousarray(v)) for k, v in state.items()}
    dec.load_state_dict(sd)
    dec.eval()
    return dec


def make_optimizer(dec, optim_cfg, data_type="KITTI"):
    ref = load()
    cfg = ref.utils.ForceKeyErrorDict(data_type=data_type, optimizer=optim_cfg)
    return ref.optimizer.Optimizer(dec, cfg)

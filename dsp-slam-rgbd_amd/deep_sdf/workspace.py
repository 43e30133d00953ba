"""DeepSDF checkpoint loader — the weight-format boundary of the hot path.

Replaces ``deep_sdf/workspace.py:202-223`` (``config_decoder``): reads the same
``specs.json`` + ``ModelParameters/<checkpoint>.pth`` (``model_state_dict`` with
``module.lin{i}.weight_g / weight_v / bias`` keys, workspace.py:214-218), folds
weight normalisation exactly as the reference module does at forward time
(``torch._weight_norm(v, g, 0)``, i.e. ``nn.utils.weight_norm``'s hook) so the
effective fp32 weights are bit-identical, and uploads them once into libdsr's
MFMA fragment layout.  The checkpoint is read with ``torch.load(weights_only=True)``
only.  PyTorch is plumbing here (file format + the fold), never compute.
"""
from __future__ import annotations

import json
import os

import numpy as np

model_params_subdir = "ModelParameters"
specifications_filename = "specs.json"


def load_specs(experiment_directory):
    fn = os.path.join(experiment_directory, specifications_filename)
    if not os.path.isfile(fn):
        raise Exception('The experiment directory does not include specifications file "specs.json"')
    with open(fn) as f:
        return json.load(f)


def fold_state(state_dict, specs):
    """Effective (W, b) per ``lin{i}`` as fp32 numpy arrays, computed with torch's own
    weight-norm op (same kernel the reference's hook runs)."""
    import torch

    sd = {}
    for k, v in state_dict.items():
        k = k[len("module."):] if k.startswith("module.") else k
        sd[k] = v if isinstance(v, torch.Tensor) else torch.from_numpy(np.asarray(v))
    layers = []
    i = 0
    while f"lin{i}.bias" in sd:
        if f"lin{i}.weight_v" in sd:
            W = torch._weight_norm(sd[f"lin{i}.weight_v"].float(), sd[f"lin{i}.weight_g"].float(), 0)
        else:
            W = sd[f"lin{i}.weight"].float()
        layers.append((W.detach().cpu().numpy().astype(np.float32),
                       sd[f"lin{i}.bias"].float().detach().cpu().numpy().astype(np.float32)))
        i += 1
    if not layers:
        raise ValueError("checkpoint holds no lin{i} layers")
    return layers


def norm_state(state_dict, specs):
    """LayerNorm parameters per ``lin{j}`` (j = 0..7): ``(gamma, beta)`` fp32 arrays where
    deep_sdf_decoder.py:58-63 builds ``bn{j} = nn.LayerNorm(out_dim)`` (weight_norm=False and
    j in norm_layers; applied between lin{j} and its ReLU, :96-102), else None."""
    ns = specs["NetworkSpecs"]
    out = [None] * 8
    if ns.get("weight_norm", False):
        return out
    sd = {(k[len("module."):] if k.startswith("module.") else k): v for k, v in state_dict.items()}
    for j in range(8):
        if j in (ns.get("norm_layers") or ()):
            if f"bn{j}.weight" not in sd or f"bn{j}.bias" not in sd:
                raise ValueError(f"checkpoint lacks bn{j}.weight / bn{j}.bias for its LayerNorm")
            out[j] = tuple(np.asarray(sd[f"bn{j}.{k}"].detach().cpu().numpy() if hasattr(sd[f"bn{j}.{k}"], "detach")
                                      else sd[f"bn{j}.{k}"], np.float32).reshape(-1) for k in ("weight", "bias"))
    return out


def check_topology(specs, layers):
    """Reject decoder variants libdsr does not implement (loudly, never approximated): other dims
    / latent_in / CodeLength.  Implemented: use_tanh, xyz_in_all and LayerNorm layers
    (weight_norm=False with norm_layers: norm_state) on the split-fp16 kernels, never the lite
    pass; plain Linear layers (fold_state reads their ``weight``); dropout / latent_dropout, which
    are identities in eval mode (deep_sdf_decoder.py:78-83, :104-105)."""
    ns = specs["NetworkSpecs"]
    if list(ns.get("latent_in", [])) != [4]:
        raise NotImplementedError("libdsr supports latent_in=[4] only")
    if list(ns.get("dims", [512] * 8)) != [512] * 8:
        raise NotImplementedError("libdsr supports dims=[512]*8 only")
    L = specs["CodeLength"]
    if L not in (64, 32):
        raise NotImplementedError("libdsr supports CodeLength 64 or 32")
    # deep_sdf_decoder.py:41-47: xyz_in_all takes 3 outputs off every hidden layer but lin3
    h = 509 if ns.get("xyz_in_all") else 512
    shapes = [W.shape for W, _ in layers]
    want = [(h, L + 3)] + [(h, 512)] * 2 + [(509 - L, 512)] + [(h, 512)] * 4 + [(1, 512)]
    if shapes != want:
        raise NotImplementedError(f"unsupported decoder shapes {shapes}")


class Decoder:
    """Device-resident DeepSDF decoder handle (what ``get_decoder`` returns).

    Mirrors what the reference's callers use of the module: it is passed to
    ``Optimizer`` / ``MeshExtractor``; ``code_len`` and ``layers`` are informative.
    """

    def __init__(self, specs, layers, device=None, ctx=None, norms=None):
        import ctypes as C

        from reconstruct import _libdsr as L

        check_topology(specs, layers)
        norms = list(norms) if norms is not None else [None] * 8
        if any(n is not None for n in norms) and specs["NetworkSpecs"].get("weight_norm", False):
            raise ValueError("LayerNorm parameters given for a weight-normed decoder")
        for j, n in enumerate(norms):
            if n is not None and (n[0].shape != (layers[j][0].shape[0],) or n[1].shape != n[0].shape):
                raise NotImplementedError(f"bn{j} shapes {n[0].shape} / {n[1].shape} do not match lin{j}")
        self.specs = specs
        self.code_len = specs["CodeLength"]
        self.layers = layers
        self.ctx = ctx if ctx is not None else L.Context.get(device)   # ctx: an explicit context
        desc = L.DecoderDesc()
        desc.code_len = self.code_len
        desc.n_layers = len(layers)
        for i, (W, _) in enumerate(layers):
            desc.out_dim[i], desc.in_dim[i] = W.shape
        desc.latent_in = 4
        ns = specs["NetworkSpecs"]
        desc.use_tanh = 1 if ns.get("use_tanh") else 0          # deep_sdf_decoder.py:65-67, :93-94
        desc.xyz_in_all = 1 if ns.get("xyz_in_all") else 0      # :46-47, :89-90
        desc.norm_mask = sum(1 << j for j, n in enumerate(norms) if n is not None)   # :58-63, :96-102
        flat = np.concatenate([np.concatenate([W.reshape(-1), b.reshape(-1)]) for W, b in layers] +
                              [np.concatenate([n[0], n[1]]) for n in norms if n is not None])
        self._flat = np.ascontiguousarray(flat, np.float32)
        h = C.c_void_p()
        self.ctx.check(self.ctx.lib.dsr_decoder_load(self.ctx.handle, C.byref(desc),
                                                     L.fptr(self._flat), self._flat.size,
                                                     C.byref(h)), "dsr_decoder_load")
        self.handle = h

    @property
    def info(self):
        """The load-time lite qualification (dsr_decoder_info_get) as a dict:
        ``lite_eligible`` False means every batch on this decoder decodes exactly."""
        import ctypes as C

        from reconstruct import _libdsr as L

        inf = L.DecoderInfo()
        self.ctx.check(self.ctx.lib.dsr_decoder_info_get(self.handle, C.byref(inf)), "dsr_decoder_info_get")
        d = {k: getattr(inf, k) for k, _ in inf._fields_}
        d["lite_eligible"] = bool(d["lite_eligible"])
        return d

    def __del__(self):
        try:
            if getattr(self, "handle", None):
                self.ctx.lib.dsr_decoder_free(self.ctx.handle, self.handle)
                self.handle = None
        except Exception:
            pass


def decoder_from_state(state_dict, specs, device=None):
    return Decoder(specs, fold_state(state_dict, specs), device, norms=norm_state(state_dict, specs))


def config_decoder(experiment_directory, checkpoint="latest", device=None):
    """workspace.py:202-223: specs.json + ModelParameters/<checkpoint>.pth -> decoder."""
    import torch

    specs = load_specs(experiment_directory)
    if specs.get("NetworkArch", "deep_sdf_decoder") != "deep_sdf_decoder":
        raise NotImplementedError("only NetworkArch=deep_sdf_decoder is supported")
    saved = torch.load(os.path.join(experiment_directory, model_params_subdir, checkpoint + ".pth"),
                       map_location="cpu", weights_only=True)
    return decoder_from_state(saved["model_state_dict"], specs, device)

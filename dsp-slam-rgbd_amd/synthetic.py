"""Seeded synthetic workloads for the DeepSDF shape-prior reconstruction path.

The reference's DeepSDF weights (``weights/deepsdf/{cars_64,chairs_64}``) and
its KITTI / Redwood data are not available offline, so tests,
golden fixtures and ``bench.py`` all run on the workload defined here
(SURVEY.md §8d):

* a DeepSDF 8x512 decoder in the reference's checkpoint format
  (``deep_sdf/workspace.py:202-223`` loads ``module.lin{i}.weight_g / weight_v
  / bias``): PyTorch-Linear-like U(+-1/sqrt(fan_in)) init, hidden layers x2.45
  so activation scale survives the ReLUs, code columns of lin0/lin4 x0.1 (a
  code of norm ~1 moves the surface by a few cm, like a trained DeepSDF), and
  the last layer least-squares fitted (ridge, fp64) so that at code 0 the
  decoder is a unit-gradient SDF of the r=0.5 sphere with ~4e-3 rms wiggles —
  i.e. it behaves like a trained DeepSDF (thin |sdf|<0.01 band, K ~ 1-2 render
  points per foreground ray) instead of a random function;
* objects shaped like ``kitti_sequence.py:141-146, 203-210`` hands them to
  ``Optimizer.reconstruct_object`` (``optimizer.py:90``): N surface points,
  N foreground rays (one per surface point) + 200 background rays, N depths.

Everything is numpy + json; nothing here imports torch (the checkpoint writer
does, lazily) so the generator runs identically on the GPU box and here.
"""
from __future__ import annotations

import hashlib
import json
import os
from dataclasses import dataclass

import numpy as np

#: DeepSDF ``specs.json`` NetworkSpecs used by DSP-SLAM's cars_64 / chairs_64
#: decoders (upstream DeepSDF defaults, SURVEY.md §8c "Weights").
DEFAULT_SPECS = {
    "NetworkArch": "deep_sdf_decoder",
    "CodeLength": 64,
    "NetworkSpecs": {
        "dims": [512, 512, 512, 512, 512, 512, 512, 512],
        "dropout": [0, 1, 2, 3, 4, 5, 6, 7],
        "dropout_prob": 0.2,
        "norm_layers": [0, 1, 2, 3, 4, 5, 6, 7],
        "latent_in": [4],
        "xyz_in_all": False,
        "use_tanh": False,
        "latent_dropout": False,
        "weight_norm": True,
    },
}

#: optimizer blocks of configs/config_kitti.json:21-39 and
#: configs/config_redwood_01053.json:15-30 (the two BASELINE parameter sets).
KITTI_OPTIM = {
    "code_len": 64, "num_depth_samples": 50, "cut_off_threshold": 0.01,
    "joint_optim": {"k1": 1.0, "k2": 100.0, "k3": 0.25, "k4": 1e7, "b1": 0.20,
                    "b2": 0.025, "num_iterations": 10, "learning_rate": 1.0,
                    "scale_damping": 1.0},
    "pose_only_optim": {"num_iterations": 5, "learning_rate": 1.0},
}
REDWOOD_OPTIM = {
    "code_len": 64, "num_depth_samples": 50, "cut_off_threshold": 0.01,
    "joint_optim": {"k1": 10.0, "k2": 100.0, "k3": 2.5, "k4": 0.0, "b1": 0.20,
                    "b2": 0.02, "num_iterations": 5, "learning_rate": 1.0,
                    "scale_damping": 100.0},
}


def layer_shapes(specs=DEFAULT_SPECS):
    """(out, in) of every ``lin{i}`` exactly as deep_sdf_decoder.py:29-56 builds them."""
    L = specs["CodeLength"]
    ns = specs["NetworkSpecs"]
    dims = [L + 3] + list(ns["dims"]) + [1]
    latent_in = ns.get("latent_in", ())
    shapes = []
    for layer in range(len(dims) - 1):
        if layer + 1 in latent_in:
            out_dim = dims[layer + 1] - dims[0]
        else:
            out_dim = dims[layer + 1]
            if ns.get("xyz_in_all") and layer != len(dims) - 2:
                out_dim -= 3
        shapes.append((out_dim, dims[layer]))
    return shapes


def make_decoder_state(seed: int = 1234, specs=DEFAULT_SPECS, hidden_gain=2.45,
                       last_gain=10.0, code_gain=0.1):
    """Return an OrderedDict-like ``{name: np.float32 array}`` in checkpoint format.

    Names carry the ``module.`` prefix the reference's DataParallel wrapper
    expects (workspace.py:214-218).  The last bias is shifted afterwards by
    :func:`calibrate_last_bias`, which needs a forward pass.
    """
    rng = np.random.default_rng(seed)
    ns = specs["NetworkSpecs"]
    shapes = layer_shapes(specs)
    n = len(shapes)
    state = {}
    for layer, (out_dim, in_dim) in enumerate(shapes):
        bound = 1.0 / np.sqrt(in_dim)
        v = rng.uniform(-bound, bound, size=(out_dim, in_dim))
        b = rng.uniform(-bound, bound, size=(out_dim,))
        if layer == n - 1:
            v *= last_gain
        elif layer > 0:
            v *= hidden_gain
        else:
            v *= hidden_gain * 2.0
        L = specs["CodeLength"]
        if layer == 0:
            v[:, :L] *= code_gain
        if layer in ns.get("latent_in", ()):
            v[:, in_dim - (L + 3):in_dim - 3] *= code_gain
        name = f"module.lin{layer}"
        if ns.get("weight_norm") and layer in ns.get("norm_layers", ()):
            g = np.linalg.norm(v, axis=1, keepdims=True) * rng.uniform(0.9, 1.1, size=(out_dim, 1))
            state[name + ".weight_g"] = g.astype(np.float32)
            state[name + ".weight_v"] = v.astype(np.float32)
        else:
            state[name + ".weight"] = v.astype(np.float32)
        state[name + ".bias"] = b.astype(np.float32)
        if not ns.get("weight_norm") and layer in (ns.get("norm_layers") or ()) and layer < n - 1:
            # nn.LayerNorm(out_dim) between lin{layer} and its ReLU (deep_sdf_decoder.py:58-63)
            state[f"module.bn{layer}.weight"] = rng.uniform(0.8, 1.2, size=(out_dim,)).astype(np.float32)
            state[f"module.bn{layer}.bias"] = rng.uniform(-0.1, 0.1, size=(out_dim,)).astype(np.float32)
    return state


def _norms_np(state, specs):
    """LayerNorm (gamma, beta) per hidden layer (None where there is none), fp64."""
    ns = specs["NetworkSpecs"]
    out = []
    for j in range(len(layer_shapes(specs)) - 1):
        k = f"module.bn{j}.weight"
        out.append((state[k].astype(np.float64), state[f"module.bn{j}.bias"].astype(np.float64))
                   if (not ns.get("weight_norm") and k in state) else None)
    return out


def _ln_f64(x, gb):
    mu = x.mean(-1, keepdims=True)
    var = ((x - mu) ** 2).mean(-1, keepdims=True)
    return (x - mu) / np.sqrt(var + 1e-5) * gb[0] + gb[1]


def fold_weight_norm_np(state, specs=DEFAULT_SPECS):
    """Effective (W, b) per layer, W = v * (g / ||v||_row) (torch._weight_norm, dim=0).

    float64 fold rounded to fp32 — only used for calibration / statistics; the
    device loader folds with torch itself so W is bit-identical to the
    reference module's."""
    layers = []
    for layer in range(len(layer_shapes(specs))):
        name = f"module.lin{layer}"
        if name + ".weight_v" in state:
            v = state[name + ".weight_v"].astype(np.float64)
            g = state[name + ".weight_g"].astype(np.float64)
            W = v * (g / np.linalg.norm(v, axis=1, keepdims=True))
        else:
            W = state[name + ".weight"].astype(np.float64)
        layers.append((W.astype(np.float32), state[name + ".bias"].astype(np.float32)))
    return layers


def _forward_f64(layers, inp, latent_in=(4,), xyz_in_all=False, norms=None):
    """Pre-tanh output (deep_sdf_decoder.py:75-103: latent skip, xyz_in_all concat, LayerNorm, ReLU)."""
    x = _features_f64(layers, inp, latent_in, xyz_in_all, norms)
    W, b = layers[-1]
    return (x @ W.T.astype(np.float64) + b)[..., 0]


def calibrate_last_bias(state, specs=DEFAULT_SPECS, seed=99, n=4096, radius=0.5):
    """Shift the last bias so the median pre-tanh output on the r=0.5 shell at z=0 is 0."""
    rng = np.random.default_rng(seed)
    p = rng.standard_normal((n, 3))
    p = radius * p / np.linalg.norm(p, axis=1, keepdims=True)
    L = specs["CodeLength"]
    inp = np.concatenate([np.zeros((n, L)), p], axis=1)
    layers = fold_weight_norm_np(state, specs)
    ns = specs["NetworkSpecs"]
    pre = _forward_f64(layers, inp, tuple(ns.get("latent_in", ())), bool(ns.get("xyz_in_all")),
                       _norms_np(state, specs))
    last = f"module.lin{len(layers) - 1}.bias"
    state[last] = (state[last].astype(np.float64) - np.median(pre)).astype(np.float32)
    return state


def _features_f64(layers, inp, latent_in=(4,), xyz_in_all=False, norms=None):
    """The last layer's input: hidden features (+ xyz under xyz_in_all)."""
    x = inp
    n = len(layers)
    for i, (W, b) in enumerate(layers[:-1]):
        if i in latent_in:
            x = np.concatenate([x, inp], axis=-1)
        elif i != 0 and xyz_in_all:
            x = np.concatenate([x, inp[..., -3:]], axis=-1)
        x = x @ W.T.astype(np.float64) + b
        if norms is not None and norms[i] is not None:
            x = _ln_f64(x, norms[i])
        x = np.maximum(x, 0.0)
    if n - 1 in latent_in:
        x = np.concatenate([x, inp], axis=-1)
    elif xyz_in_all:
        x = np.concatenate([x, inp[..., -3:]], axis=-1)
    return x


def fit_last_layer_to_sphere(state, specs=DEFAULT_SPECS, seed=5, n=12000, radius=0.5, lam=1e-3):
    """Ridge-fit lin{last} so pre-tanh(x) ~= |x| - radius at code 0 (fp64, deterministic)."""
    rng = np.random.default_rng(seed)
    d = rng.standard_normal((n, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    r = np.concatenate([rng.uniform(0, 1, n // 2) ** (1 / 3),
                        radius + 0.08 * rng.standard_normal(n - n // 2)])
    x = d * r[:, None]
    L = specs["CodeLength"]
    inp = np.concatenate([np.zeros((n, L)), x], axis=1)
    layers = fold_weight_norm_np(state, specs)
    ns = specs["NetworkSpecs"]
    H = _features_f64(layers, inp, tuple(ns.get("latent_in", ())), bool(ns.get("xyz_in_all")),
                      _norms_np(state, specs))
    A = np.concatenate([H, np.ones((n, 1))], axis=1)
    tgt = np.linalg.norm(x, axis=1) - radius
    w = np.linalg.solve(A.T @ A + lam * np.eye(A.shape[1]), A.T @ tgt)
    last = len(layers) - 1
    name = f"module.lin{last}"
    state[name + ".weight"] = w[None, :-1].astype(np.float32)
    state[name + ".bias"] = np.array([w[-1]], np.float32)
    return state


def make_decoder(seed: int = 1234, specs=DEFAULT_SPECS):
    return fit_last_layer_to_sphere(make_decoder_state(seed, specs), specs)


def state_sha256(state) -> str:
    h = hashlib.sha256()
    for k in sorted(state):
        h.update(k.encode())
        h.update(np.ascontiguousarray(state[k], dtype=np.float32).tobytes())
    return h.hexdigest()


def write_experiment_dir(path, state, specs=DEFAULT_SPECS, checkpoint="latest"):
    """Write ``specs.json`` + ``ModelParameters/<checkpoint>.pth`` like a DeepSDF run.

    The .pth holds ``{"epoch": 0, "model_state_dict": {...torch tensors...}}``
    (workspace.py:215-218), readable with ``torch.load(weights_only=True)``.
    """
    import torch  # lazy: only the checkpoint writer needs torch

    os.makedirs(os.path.join(path, "ModelParameters"), exist_ok=True)
    with open(os.path.join(path, "specs.json"), "w") as f:
        json.dump(specs, f, indent=2)
    sd = {k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in state.items()}
    torch.save({"epoch": 0, "model_state_dict": sd},
               os.path.join(path, "ModelParameters", checkpoint + ".pth"))
    return path


@dataclass
class SyntheticObject:
    t_cam_obj: np.ndarray   # (4,4) f32 initial object->camera Sim(3)
    pts: np.ndarray         # (N,3) f32 surface points, camera frame
    rays: np.ndarray        # (N+n_bg,3) f32 ray directions (fg first, then bg)
    depth: np.ndarray       # (N,) f32 observed depth of fg rays
    t_true: np.ndarray      # (4,4) f32 the pose the points were generated with


def _rot_y(theta):
    c, s = np.cos(theta), np.sin(theta)
    return np.array([[c, 0, s], [0, 1, 0], [-s, 0, c]])


def make_object(seed: int, n_pts: int = 2048, n_bg: int = 200, scale: float = 2.0,
                tz: float = 15.0, upright: bool = True, perturb: float = 1.0,
                radius: float = 0.5) -> SyntheticObject:
    """One synthetic instance (SURVEY.md §8d "Synthetic object").

    Surface points 0.5*normalize(N(0,I)) in the object frame; pose
    R = diag(1,-1,-1) R_y(theta) (camera y down, object upright for the KITTI
    rotation prior), scale ``scale``, translation (0,0,tz).  Foreground rays are
    pts_cam / z (kitti_sequence.py:203-210 builds rays from the projected
    pixels, fg first), background rays (u,v,1) with u,v ~ U(+-0.6 s/tz).  The
    initial pose handed to the optimizer is the true pose perturbed by a few
    degrees / centimetres / percent (``perturb`` scales it; 0 = exact).
    """
    rng = np.random.default_rng(seed)
    p = rng.standard_normal((n_pts, 3))
    p = radius * p / np.linalg.norm(p, axis=1, keepdims=True)
    theta = rng.uniform(-np.pi, np.pi)
    R = (np.diag([1.0, -1.0, -1.0]) if upright else np.eye(3)) @ _rot_y(theta)
    t = np.array([0.0, 0.0, tz])
    pts_cam = scale * p @ R.T + t
    fg = pts_cam / pts_cam[:, 2:3]
    span = 0.6 * scale / tz
    bg = np.stack([rng.uniform(-span, span, n_bg), rng.uniform(-span, span, n_bg),
                   np.ones(n_bg)], axis=1)
    rays = np.concatenate([fg, bg], axis=0)
    T = np.eye(4)
    T[:3, :3] = scale * R
    T[:3, 3] = t
    # perturbation: small yaw, translation and scale error
    dth = perturb * rng.uniform(-0.05, 0.05)
    dt = perturb * rng.uniform(-0.05, 0.05, size=3)
    ds = 1.0 + perturb * rng.uniform(-0.03, 0.03)
    T0 = np.eye(4)
    T0[:3, :3] = ds * scale * R @ _rot_y(dth)
    T0[:3, 3] = t + dt
    return SyntheticObject(
        t_cam_obj=T0.astype(np.float32),
        pts=pts_cam.astype(np.float32),
        rays=rays.astype(np.float32),
        depth=pts_cam[:, 2].astype(np.float32),
        t_true=T.astype(np.float32),
    )


def kitti_object(obj_id: int, base_seed: int = 1000, n_pts: int = 2048):
    """Metric-unit object (config 2): KITTI params, 2048 pts, 2048+200 rays, s=2, tz=15."""
    return make_object(base_seed + obj_id, n_pts=n_pts, scale=2.0, tz=15.0, upright=True)


def redwood_object(obj_id: int, base_seed: int = 2000, n_pts: int = 512):
    """Config 1 shape: Redwood params, 512 pts, 512+200 rays, R=I-ish, s=1, tz=3."""
    return make_object(base_seed + obj_id, n_pts=n_pts, scale=1.0, tz=3.0, upright=False)

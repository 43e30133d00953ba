"""CPU oracle for the DeepSDF shape-prior reconstruction hot path.

TEST INFRASTRUCTURE ONLY.  This module is the *checker*: only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
it.  The product path (``dsp-slam-rgbd_amd/reconstruct`` -> ``libdsr.so``) never
calls into it and fails loudly when the HIP library is missing.

It is a from-scratch numpy restatement of the reference's algorithm (the
reference is PyTorch; nothing here imports torch or the reference).  Every
function cites the reference ``file:line`` it restates.  Arithmetic is fp32 by
default (the reference's dtype) and can be run in fp64 (``dtype=np.float64``)
as a "truth" to measure how far fp32 implementations drift.

Pinning: the restatement is checked against golden vectors produced by
importing the reference itself in the build container
(``tests/golden/make_golden.py`` -> ``tests/golden/*.npz``, tests in
``tests/test_oracle_golden.py``).  Where the reference's own result depends on
fp32 summation order (CPU thread count), the fixtures record that spread and the
tests use it as the noise floor.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import numpy as np

F32 = np.float32


# --------------------------------------------------------------------------------------
# decoder (deep_sdf/deep_sdf_decoder.py)
# --------------------------------------------------------------------------------------
class Decoder:
    """DeepSDF MLP, eval mode (deep_sdf_decoder.py:10-110).

    ``layers`` are the *effective* (W, b) per ``lin{i}`` (weight-norm already
    folded, W = v * (g / ||v||), deep_sdf_decoder.py:49-53).  Dropout and latent
    dropout are inert in eval (:78-83, :104-105).  Variants: ``xyz_in_all`` (every
    layer's input but lin0's and the latent-skip layer's gets xyz appended, :89-90),
    ``use_tanh`` (a tanh after the last layer, before the final ``self.th``, :93-94) and
    LayerNorm (``norms[i] = (gamma, beta)``: nn.LayerNorm between lin{i} and its ReLU,
    :58-63, :96-102, eps 1e-5, biased variance); the final ``self.th`` tanh (:72,
    :107-108) is always applied.
    """

    def __init__(self, layers, code_len=64, latent_in=(4,), dtype=F32, xyz_in_all=False, use_tanh=False,
                 norms=None):
        self.dtype = dtype
        self.layers = [(np.asarray(W, dtype), np.asarray(b, dtype)) for W, b in layers]
        self.code_len = code_len
        self.latent_in = tuple(latent_in)
        self.xyz_in_all = bool(xyz_in_all)
        self.use_tanh = bool(use_tanh)
        self.norms = [None if n is None else (np.asarray(n[0], dtype), np.asarray(n[1], dtype))
                      for n in (norms or [None] * len(self.layers))]

    @classmethod
    def from_state(cls, state, specs, dtype=F32):
        """Fold a ``module.lin{i}.weight_g/_v/bias`` state dict (workspace.py:214-218)."""
        ns = specs["NetworkSpecs"]
        norms = [None] * 9
        if not ns.get("weight_norm"):
            for j in range(8):
                if j in (ns.get("norm_layers") or ()) and f"module.bn{j}.weight" in state:
                    norms[j] = (np.asarray(state[f"module.bn{j}.weight"], np.float32),
                                np.asarray(state[f"module.bn{j}.bias"], np.float32))
        layers = []
        i = 0
        while f"module.lin{i}.bias" in state:
            name = f"module.lin{i}"
            if name + ".weight_v" in state:
                v = np.asarray(state[name + ".weight_v"], np.float32)
                g = np.asarray(state[name + ".weight_g"], np.float32)
                nrm = np.sqrt((v.astype(np.float64) ** 2).sum(1, keepdims=True)).astype(np.float32)
                W = v * (g / nrm)
            else:
                W = np.asarray(state[name + ".weight"], np.float32)
            layers.append((W, np.asarray(state[name + ".bias"], np.float32)))
            i += 1
        return cls(layers, specs["CodeLength"], ns.get("latent_in", ()), dtype,
                   bool(ns.get("xyz_in_all")), bool(ns.get("use_tanh")), norms[:len(layers)])

    def _ln(self, x, i, keep):
        """nn.LayerNorm (deep_sdf_decoder.py:96-101): (x - mean) / sqrt(var + eps) * gamma + beta."""
        g, b = self.norms[i]
        mu = x.mean(-1, keepdims=True, dtype=self.dtype)
        d = x - mu
        rstd = self.dtype(1) / np.sqrt((d * d).mean(-1, keepdims=True, dtype=self.dtype) + self.dtype(1e-5))
        xh = d * rstd
        if keep is not None:
            keep[i] = (xh, rstd)
        return xh * g + b

    def forward(self, inp, keep_masks=False, keep_pre=False, keep_ln=None):
        """inp (n, L+3) -> sdf (n,).  deep_sdf_decoder.py:75-110."""
        inp = np.asarray(inp, self.dtype)
        xyz = inp[..., -3:]
        x = inp
        masks = []
        n_layers = len(self.layers)
        for i, (W, b) in enumerate(self.layers):
            if i in self.latent_in:
                x = np.concatenate([x, inp], axis=-1)          # :87-88
            elif i != 0 and self.xyz_in_all:
                x = np.concatenate([x, xyz], axis=-1)          # :89-90
            x = x @ W.T + b                                    # :91
            if i == n_layers - 1 and self.use_tanh:
                x = np.tanh(x)                                 # :93-94
            if i < n_layers - 1:
                if self.norms[i] is not None:
                    x = self._ln(x, i, keep_ln)                # :96-101
                m = x > 0
                x = np.where(m, x, self.dtype(0))              # :103 ReLU
                if keep_masks:
                    masks.append(m)
        t = x[..., 0]
        y = np.tanh(t)                                         # :107-108 self.th
        if keep_pre:
            return y, masks, t
        return (y, masks) if keep_masks else y

    def forward_jac(self, inp):
        """(y, dy/dinp) — what ``get_batch_sdf_jacobian`` (loss_utils.py:82-113) gets
        from autograd, restated as the analytic chain rule:
        tanh' = 1-y^2 (use_tanh: times 1-t^2 of the inner tanh), ReLU' = [out>0],
        Linear' = W^T, latent-skip split at layer 4, xyz_in_all columns to d/dxyz."""
        inp = np.asarray(inp, self.dtype)
        lnk = {}
        y, masks, t = self.forward(inp, keep_masks=True, keep_pre=True, keep_ln=lnk)
        n_layers = len(self.layers)
        L3 = inp.shape[-1]
        g = (self.dtype(1) - y * y)[:, None]                   # d tanh
        if self.use_tanh:
            g = g * (self.dtype(1) - t * t)[:, None]           # d tanh of the use_tanh layer
        grad_in = np.zeros_like(inp)
        for i in range(n_layers - 1, -1, -1):
            W, _ = self.layers[i]
            if i < n_layers - 1 and i in lnk:                  # through lin{i}'s LayerNorm
                xh, rstd = lnk[i]
                gx = g * self.norms[i][0]
                g = rstd * (gx - gx.mean(-1, keepdims=True, dtype=self.dtype)
                            - xh * (gx * xh).mean(-1, keepdims=True, dtype=self.dtype))
            g = g @ W                                          # d/d(input of layer i)
            if i in self.latent_in:
                grad_in = grad_in + g[:, -L3:]
                g = g[:, :-L3]
            elif i != 0 and self.xyz_in_all:
                grad_in[:, -3:] = grad_in[:, -3:] + g[:, -3:]
                g = g[:, :-3]
            if i > 0:
                g = np.where(masks[i - 1], g, self.dtype(0))
        grad_in = g + grad_in                                  # layer-0 path + skip path
        return y, grad_in


# --------------------------------------------------------------------------------------
# loss_utils.py
# --------------------------------------------------------------------------------------
def sdf_to_occupancy(sdf, th):
    """loss_utils.py:40-48: 0.5 - clamp(sdf,+-th)/(2 th)."""
    dt = sdf.dtype.type
    return dt(0.5) - np.clip(sdf, dt(-th), dt(th)) / dt(2 * th)


def decode_sdf(dec: Decoder, z, x, max_batch=64 ** 3):
    """loss_utils.py:51-79 — no-grad forward with the code broadcast, chunked."""
    out = []
    for h in range(0, x.shape[0], max_batch):
        xs = x[h:h + max_batch, :3]
        inp = np.concatenate([np.broadcast_to(z, (xs.shape[0], z.shape[0])), xs], axis=-1)
        out.append(dec.forward(inp))
    return np.concatenate(out) if out else np.zeros(0, dec.dtype)


def get_batch_sdf_jacobian(dec: Decoder, z, x):
    """loss_utils.py:82-113 — returns sdf (n,) and d sdf / d[code, xyz] (n, L+3)."""
    inp = np.concatenate([np.broadcast_to(z, (x.shape[0], z.shape[0])), x], axis=-1)
    return dec.forward_jac(inp)


def neg_hat(p):
    """-[p]x per point, the ``negate_hat`` block of loss_utils.py:117-136 / :176-195."""
    x, y, zz = p[:, 0], p[:, 1], p[:, 2]
    zero = np.zeros_like(x)
    cols = [np.stack([zero, -zz, y], -1), np.stack([zz, zero, -x], -1), np.stack([-y, x, zero], -1)]
    return np.stack(cols, axis=-1)          # stack on dim=-1: the lists are COLUMNS


def get_points_to_pose_jacobian_se3(p):
    """loss_utils.py:117-136: [I | -[p]x] (n,3,6)."""
    eye = np.broadcast_to(np.eye(3, dtype=p.dtype), (p.shape[0], 3, 3))
    return np.concatenate([eye, neg_hat(p)], axis=-1)


def get_points_to_pose_jacobian_sim3(p):
    """loss_utils.py:176-195: [I | -[p]x | p] (n,3,7)."""
    return np.concatenate([get_points_to_pose_jacobian_se3(p), p[..., None]], axis=-1)


def _hat(w):
    dt = w.dtype.type
    return np.array([[0., -w[2], w[1]], [w[2], 0., -w[0]], [-w[1], w[0], 0.]], dtype=dt)


def exp_se3(x):
    """loss_utils.py:139-173 (translation first, then rotation)."""
    dt = x.dtype.type
    v, w = x[:3], x[3:6]
    W = _hat(w)
    W2 = W @ W
    theta = dt(np.sqrt(np.sum(w * w)))
    eye = np.eye(3, dtype=x.dtype)
    if theta <= 1e-8:
        e_w, j = eye, eye
    else:
        st, ct = dt(np.sin(theta)), dt(np.cos(theta))
        t2, t3 = theta * theta, theta * theta * theta
        e_w = eye + W * st / theta + W2 * (dt(1) - ct) / t2
        k1 = (dt(1) - ct) / t2
        k2 = (theta - st) / t3
        j = eye + k1 * W + k2 * W2
    out = np.eye(4, dtype=x.dtype)
    out[:3, :3] = e_w
    out[:3, 3] = j @ v
    return out


def exp_sim3(x):
    """loss_utils.py:198-243, branch structure included: theta<=1e-8 with s==0 /
    s!=0, and the reference's ``c = 0 if s <= eps`` (also for NEGATIVE s) quirk."""
    dt = x.dtype.type
    v, w, s = x[:3], x[3:6], x[6]
    W = _hat(w)
    W2 = W @ W
    theta = dt(np.sqrt(np.sum(w * w)))
    t2 = theta * theta
    st, ct = dt(np.sin(theta)), dt(np.cos(theta))
    e_s = dt(np.exp(s))
    s2 = s * s
    eye = np.eye(3, dtype=x.dtype)
    eps = 1e-8
    if theta <= 1e-8:
        if s == 0:
            e_w, j = eye, eye
        else:
            e_w = eye
            j = ((e_s - dt(1)) / s) * eye
    else:
        e_w = eye + W * st / theta + W2 * (dt(1) - ct) / t2
        a = e_s * st
        b = e_s * ct
        c = dt(0) if s <= eps else (e_s - dt(1)) / s
        k0 = c * eye
        k1 = (a * s + (dt(1) - b) * theta) / (s2 + t2)
        k2 = c - ((b - dt(1)) * s + a * theta) / (s2 + t2)
        j = k0 + k1 * W / theta + k2 * W2 / t2
    out = np.eye(4, dtype=x.dtype)
    out[:3, :3] = e_s * e_w
    out[:3, 3] = j @ v
    return out


def huber_norm_weights(x, b):
    """loss_utils.py:246-257: w = sqrt(huber(|r|))/|r|, |r|==0 -> w=0."""
    dt = x.dtype.type
    rn = np.where(x <= b, x * x, dt(2 * b) * x - dt(b * b))
    den = np.where(x == 0, dt(1), x)
    return np.sqrt(rn) / den


def get_robust_res(res, b):
    """loss_utils.py:260-275: (w*r, mean((w*r)^2), w)."""
    r = res.reshape(-1)
    w = huber_norm_weights(np.abs(r), b)
    rr = w * r
    loss = rr.dtype.type(np.mean(rr * rr)) if rr.size else rr.dtype.type(np.nan)
    return rr, loss, w


def linspace_torch(start, end, steps, dtype=F32):
    """torch.linspace on CPU fp32 (used at optimizer.py:126): step=(end-start)/(n-1),
    first half fma(step, i, start), second half fma(-step, n-1-i, end) — measured
    bit-exact against torch 2.10 in this container (the kernel is FMA-contracted)."""
    dt = np.dtype(dtype).type
    start, end = dt(start), dt(end)
    step = dt((end - start) / dt(steps - 1))
    out = np.empty(steps, dtype)
    half = steps // 2
    for i in range(steps):
        if i < half:
            out[i] = dt(np.float64(step) * i + np.float64(start))
        else:
            out[i] = dt(np.float64(end) - np.float64(step) * (steps - 1 - i))
    return out


# --------------------------------------------------------------------------------------
# loss.py
# --------------------------------------------------------------------------------------
def transform_points(p, t_obj_cam):
    """``(p[...,None,:] * T[:3,:3]).sum(-1) + T[:3,3]`` (loss.py:31-32, :74-77)."""
    R, t = t_obj_cam[:3, :3], t_obj_cam[:3, 3]
    prod = p[..., None, :] * R
    return (prod[..., 0] + prod[..., 1]) + prod[..., 2] + t


def compute_sdf_loss(dec, pts_cam, t_obj_cam, z):
    """loss.py:22-43 -> (J_pose (N,7), J_code (N,L), res (N,))."""
    x = transform_points(pts_cam, t_obj_cam)
    y, g = get_batch_sdf_jacobian(dec, z, x)
    dxo = get_points_to_pose_jacobian_sim3(x)
    j_pose = np.einsum("ni,nij->nj", g[:, -3:], dxo)
    return j_pose, g[:, :-3], y


@dataclass
class RenderOut:
    j_pose: np.ndarray
    j_code: np.ndarray
    res: np.ndarray
    n_valid: int
    ray_idx: np.ndarray
    depth_idx: np.ndarray
    pts: np.ndarray


def compute_render_loss(dec, rays, depth_obs, t_obj_cam, depths, z, th=0.01):
    """loss.py:60-166.  Returns None when fewer than 10 samples fall in the unit ball
    (:86-88).  Otherwise J/res for the K samples with |sdf|<th and de_do>1e-2."""
    dt = dec.dtype
    cam = rays[:, None, :] * depths[:, None]                         # (R, M, 3)  :71
    obj = transform_points(cam, t_obj_cam)                           # :74-77
    n_rays, n_depths = obj.shape[0], obj.shape[1]
    nrm = np.sqrt(np.sum(obj * obj, axis=-1))
    vi, vj = np.nonzero(nrm < 1.0)                                   # :82 (row-major order)
    q = obj[vi, vj]
    if q.shape[0] < 10:
        return None
    sdf = decode_sdf(dec, z, q)                                      # :91-92
    occ = np.zeros((n_rays, n_depths), dt)
    occ[vi, vj] = sdf_to_occupancy(sdf, th)                          # :97-99
    wg = (sdf > dt(-th)) & (sdf < dt(th))                            # :101
    gx, gy = vi[wg], vj[wg]
    occ_g = occ[gx, :]
    m = occ_g.shape[0]
    d_min, d_max = depths[0], depths[-1]
    acc = np.cumprod(dt(1) - occ_g, axis=-1, dtype=dt)              # :111
    acc_aug = np.concatenate([np.ones((m, 1), dt), acc], axis=-1)
    o = np.concatenate([occ_g, np.ones((m, 1), dt)], axis=-1)
    d = np.concatenate([depths, np.array([dt(1.1) * d_max], dt)])
    term = o * acc_aug
    d_u = np.sum(d * term, axis=-1)                                  # :125
    o_k = occ[gx, gy]
    l = np.arange(n_depths)[None, :]
    acc = np.where(l < gy[:, None], dt(0), acc)                      # :131
    de_do = np.sum(acc, axis=-1) / (dt(1) - o_k)
    nz = de_do > dt(1e-2)                                            # :135
    de_do, d_u = de_do[nz], d_u[nz]
    delta_d = (d_max - d_min) / dt(n_depths - 1)
    do_ds = dt(-1.0 / (2 * th))
    de_ds = de_do * delta_d * do_ds
    gx, gy = gx[nz], gy[nz]
    res = depth_obs[gx] - d_u
    res = np.clip(res, dt(-0.30), dt(0.30))                          # :147-148
    pw = obj[gx, gy]
    _, g = get_batch_sdf_jacobian(dec, z, pw)                        # :157
    de_di = de_ds[:, None] * g
    dxo = get_points_to_pose_jacobian_sim3(pw)
    j_pose = np.einsum("ni,nij->nj", de_di[:, -3:], dxo)
    return RenderOut(j_pose, de_di[:, :-3], res, int(q.shape[0]), gx, gy, pw)


def compute_rotation_loss_sim3(t_obj_cam):
    """loss.py:169-192: upright prior r = 1 - (R_co e_y).n_g, J in slots 3:6; zero when r<1e-7."""
    dt = t_obj_cam.dtype.type
    t_cam_obj = np.linalg.inv(t_obj_cam)
    r_co = t_cam_obj[:3, :3]
    scale = dt(np.linalg.det(r_co)) ** dt(1.0 / 3.0)
    r_co = r_co / scale
    r_oc = np.linalg.inv(r_co)
    ey = np.array([0., 1., 0.], t_obj_cam.dtype)
    ng = np.array([0., -1., 0.], t_obj_cam.dtype)
    ry = r_co @ ey
    res = dt(1) - np.dot(ry, ng)
    if res < 1e-7:
        return np.zeros(7, t_obj_cam.dtype), dt(0)
    jr = np.cross(r_oc @ ng, ey)
    j = np.zeros(7, t_obj_cam.dtype)
    j[3:6] = jr
    return j, res


# --------------------------------------------------------------------------------------
# optimizer.py
# --------------------------------------------------------------------------------------
@dataclass
class OptimParams:
    """Optimizer.__init__ (optimizer.py:27-43) from a configs ``optimizer`` block."""
    k1: float
    k2: float
    k3: float
    k4: float
    b1: float
    b2: float
    lr: float
    s_damp: float
    num_iterations: int
    code_len: int = 64
    num_depth_samples: int = 50
    cut_off: float = 0.01
    pose_only_iterations: int = 5

    @classmethod
    def from_cfg(cls, optim):
        jo = optim["joint_optim"]
        po = optim.get("pose_only_optim", {"num_iterations": 5})
        return cls(jo["k1"], jo["k2"], jo["k3"], jo["k4"], jo["b1"], jo["b2"],
                   jo["learning_rate"], jo["scale_damping"], jo["num_iterations"],
                   optim["code_len"], optim["num_depth_samples"], optim["cut_off_threshold"],
                   po["num_iterations"])


@dataclass
class IterTrace:
    t_obj_cam: np.ndarray
    z: np.ndarray
    loss: float
    sdf_loss: float
    render_loss: float
    n_valid: int
    k: int
    H: np.ndarray = None
    b: np.ndarray = None
    dx: np.ndarray = None


@dataclass
class ReconResult:
    t_cam_obj: np.ndarray | None
    code: np.ndarray | None
    is_good: bool
    loss: float
    trace: list = field(default_factory=list)


def gn_step(dec, p: OptimParams, t_obj_cam, z, pts, rays, depth_obs, n_fg):
    """One iteration of optimizer.py:120-194 at state (t_obj_cam, z).

    Returns (IterTrace with H/b/dx, new t_obj_cam, new z) or (IterTrace, None, None)
    on the reference's failure exits (:132-152)."""
    dt = dec.dtype
    t_cam_obj = np.linalg.inv(t_obj_cam)                               # :122
    scale = dt(np.linalg.det(t_cam_obj[:3, :3])) ** dt(1.0 / 3.0)     # :123
    d_min = t_cam_obj[2, 3] - dt(1.0) * scale
    d_max = t_cam_obj[2, 3] + dt(1.0) * scale
    depths = linspace_torch(d_min, d_max, p.num_depth_samples, dt)     # :126
    depth_obs = depth_obs.copy()
    depth_obs[n_fg:] = dt(1.1) * d_max                                 # :128
    jp_s, jc_s, r_s = compute_sdf_loss(dec, pts, t_obj_cam, z)        # :131
    rr_s, l_s, _ = get_robust_res(r_s, p.b2)
    tr = IterTrace(t_obj_cam.copy(), z.copy(), float("nan"), float(l_s), float("nan"), 0, 0)
    if math.isnan(l_s):
        return tr, None, None
    ren = compute_render_loss(dec, rays, depth_obs, t_obj_cam, depths, z, th=p.cut_off)
    if ren is None:
        return tr, None, None
    tr.n_valid, tr.k = ren.n_valid, ren.res.shape[0]
    rr_r, l_r, _ = get_robust_res(ren.res, p.b1)
    tr.render_loss = float(l_r)
    if math.isnan(l_r):
        return tr, None, None
    j_rot, r_rot = compute_rotation_loss_sim3(t_obj_cam)                # :155
    loss = dt(p.k1) * l_r + dt(p.k2) * l_s                             # :157
    tr.loss = float(loss)
    pd = 7
    J_s = np.concatenate([jp_s, jc_s], -1)
    J_r = np.concatenate([ren.j_pose, ren.j_code], -1)
    H_s = dt(p.k2) * (J_s.T @ J_s) / dt(J_s.shape[0])                  # :163
    b_s = -dt(p.k2) * (J_s.T @ rr_s) / dt(J_s.shape[0])                # :164
    H_r = dt(p.k1) * (J_r.T @ J_r) / dt(J_r.shape[0])
    b_r = -dt(p.k1) * (J_r.T @ rr_r) / dt(J_r.shape[0])
    H = H_r + H_s
    L = p.code_len
    H[pd:pd + L, pd:pd + L] += dt(p.k3) * np.eye(L, dtype=dt)           # :172
    b = b_r + b_s
    b[pd:pd + L] -= dt(p.k3) * z
    H_rot = np.outer(j_rot, j_rot)                                     # :176-181
    b_rot = -(j_rot * r_rot)
    H[:pd, :pd] += dt(p.k4) * H_rot
    b[:pd] -= dt(p.k4) * b_rot
    H[:pd, :pd] += np.eye(pd, dtype=dt)                                # :185
    H[pd - 1, pd - 1] += dt(p.s_damp)                                  # :186
    dx = np.linalg.inv(H) @ b                                          # :188
    tr.H, tr.b, tr.dx = H, b, dx
    delta_t = exp_sim3(dt(p.lr) * dx[:pd])
    t_new = delta_t @ t_obj_cam                                        # :192
    z_new = z + dt(p.lr) * dx[pd:pd + L]                               # :194
    return tr, t_new, z_new


def reconstruct_object(dec, p: OptimParams, t_cam_obj, pts, rays, depth, code=None):
    """Optimizer.reconstruct_object (optimizer.py:90-205)."""
    dt = dec.dtype
    z = np.zeros(p.code_len, dt) if code is None else np.asarray(code[:p.code_len], dt).copy()
    t_obj_cam = np.linalg.inv(np.asarray(t_cam_obj, dt))
    pts = np.asarray(pts, dt)
    rays = np.asarray(rays, dt)
    n_fg = depth.shape[0]
    depth_obs = np.concatenate([depth, np.zeros(rays.shape[0] - n_fg)]).astype(dt)
    loss = 0.0
    trace = []
    for _ in range(p.num_iterations):
        tr, t_new, z_new = gn_step(dec, p, t_obj_cam, z, pts, rays, depth_obs, n_fg)
        trace.append(tr)
        if t_new is None:
            return ReconResult(None, None, False, loss, trace)
        loss = tr.loss
        t_obj_cam, z = t_new, z_new
    return ReconResult(np.linalg.inv(t_obj_cam), z, True, loss, trace)


def estimate_pose_cam_obj(dec, p: OptimParams, t_co_se3, scale, pts, code):
    """Optimizer.estimate_pose_cam_obj (optimizer.py:46-87): SE(3) pose-only GN on
    the SDF term, H = J^T J/N + 1e-2 I, b from the UN-robustified residual."""
    dt = dec.dtype
    t_cam_obj = np.asarray(t_co_se3, dt).copy()
    t_cam_obj[:3, :3] *= dt(scale)
    t_obj_cam = np.linalg.inv(t_cam_obj)
    z = np.asarray(code, dt)
    pts = np.asarray(pts, dt)
    for e in range(p.pose_only_iterations):
        jp, _, r = compute_sdf_loss(dec, pts, t_obj_cam, z)
        j = jp[:, :6]
        hess = (j.T @ j) / dt(j.shape[0]) + dt(1e-2) * np.eye(6, dtype=dt)
        b = -(j.T @ r) / dt(j.shape[0])
        dx = np.linalg.inv(hess) @ b
        t_obj_cam = exp_se3(dx) @ t_obj_cam
        if e == 4:
            pts = pts[np.abs(r) <= 0.05]
    t_cam_obj = np.linalg.inv(t_obj_cam)
    t_cam_obj[:3, :3] /= dt(scale)
    return t_cam_obj


def compute_sdf_loss_objectpoint(dec, pts_obj, code):
    """optimizer.py:207-213 / loss.py:46-56: mean SDF of object-frame points."""
    z = np.asarray(code, dec.dtype)
    y = decode_sdf(dec, z, np.asarray(pts_obj, dec.dtype))
    return dec.dtype(np.mean(y))

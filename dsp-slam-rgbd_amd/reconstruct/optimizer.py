"""``reconstruct.optimizer`` — the Python API the C++ ORB-SLAM2 side calls (pybind11).

Same class / method names, argument meaning and return conventions as the
reference's ``reconstruct/optimizer.py``, but every numeric step
runs in libdsr's HIP kernels on an MI355X (``include/dsr.h``):

* ``Optimizer(decoder, configs)`` — optimizer.py:26-43
* ``Optimizer.reconstruct_object(t_cam_obj, pts, rays, depth, code=None)`` —
  optimizer.py:90-205 -> ``dsr_reconstruct_batch`` with one object.  Numeric
  failure returns ``is_good=False`` with ``t_cam_obj = code = None`` and ``loss``
  = the previous iteration's loss (0. if the first iteration failed), exactly
  like the reference (optimizer.py:132-152).
* ``Optimizer.reconstruct_objects([...])`` — NEW batched form: all objects of a
  keyframe / frame in one device pass.
* ``Optimizer.compute_sdf_loss_objectpoint_zhjd(pts_obj, code)`` —
  optimizer.py:207-213 -> ``dsr_sdf_eval``.
* ``Optimizer.estimate_pose_cam_obj(...)`` — optimizer.py:46-87 -> ``dsr_pose_only``.
* ``MeshExtractor`` — optimizer.py:216-233 -> ``dsr_mesher_*`` (grid decode and
  marching cubes on device).

There is no CPU fallback: without libdsr / a gfx950 device these raise DsrError.
"""
from __future__ import annotations

import ctypes as C
import os
import time

import numpy as np

from reconstruct import _libdsr as L
from reconstruct.utils import ForceKeyErrorDict, create_voxel_grid

_VERBOSE = os.environ.get("DSR_VERBOSE", "0") != "0"


def _code(code, code_len):
    """``code[:code_len]`` as a contiguous float32 vector; the C side reads exactly
    code_len floats, so a shorter array is an error, never an out-of-bounds read."""
    c = np.ascontiguousarray(np.asarray(code, np.float32).reshape(-1)[:code_len])
    if c.shape[0] != code_len:
        raise ValueError(f"code must hold at least {code_len} values, got {c.shape[0]}")
    return c


def _f32(a, shape_tail=None):
    a = np.ascontiguousarray(np.asarray(a), dtype=np.float32)
    if shape_tail is not None and (a.ndim != 2 or a.shape[1] != shape_tail):
        raise ValueError(f"expected an (N, {shape_tail}) array, got {a.shape}")
    return a


class Optimizer(object):
    def __init__(self, decoder, configs):
        self.decoder = decoder
        optim_cfg = configs.optimizer
        jo = optim_cfg.joint_optim
        self.k1 = jo.k1
        self.k2 = jo.k2
        self.k3 = jo.k3
        self.k4 = jo.k4
        self.b1 = jo.b1
        self.b2 = jo.b2
        self.lr = jo.learning_rate
        self.s_damp = jo.scale_damping
        self.num_iterations_joint_optim = jo.num_iterations
        self.code_len = optim_cfg.code_len
        self.num_depth_samples = optim_cfg.num_depth_samples
        self.cut_off = optim_cfg.cut_off_threshold
        self.num_iterations_pose_only = 5
        if configs.data_type == "KITTI":
            self.num_iterations_pose_only = optim_cfg.pose_only_optim.num_iterations
        self.params = L.OptimParams(
            float(self.k1), float(self.k2), float(self.k3), float(self.k4), float(self.b1),
            float(self.b2), float(self.lr), float(self.s_damp),
            int(self.num_iterations_joint_optim), int(self.code_len),
            int(self.num_depth_samples), float(self.cut_off), int(self.num_iterations_pose_only))
        self.last_stats = None
        # keyframe stream (BASELINE config 5): "graph" = fixed-capacity slot batches refilled per
        # keyframe, each replaying ONE captured hipGraph; "slot" = the same slots run eagerly;
        # "oneshot" = a new batch per keyframe (dsr_batch_create)
        self.keyframe_mode = os.environ.get("DSR_KEYFRAME_MODE", "graph")
        self._slots = []

    # ------------------------------------------------------------------ helpers
    @property
    def _ctx(self):
        return self.decoder.ctx

    def _object_in(self, t_cam_obj, pts, rays, depth, code, keep, pose_is_obj_cam=False):
        t = _f32(t_cam_obj).reshape(4, 4)
        pts = _f32(pts, 3)
        rays = _f32(rays, 3)
        depth = np.ascontiguousarray(np.asarray(depth, np.float32).reshape(-1))
        if depth.shape[0] > rays.shape[0]:
            raise ValueError("depth holds more values than there are rays")
        c = None if code is None else _code(code, self.code_len)
        keep.extend([pts, rays, depth, c])
        rec = L.ObjectIn()
        rec.t_cam_obj[:] = t.reshape(-1).tolist()
        rec.pts, rec.n_pts = L.fptr(pts), pts.shape[0]
        rec.rays, rec.n_rays = L.fptr(rays), rays.shape[0]
        rec.depth, rec.n_depth = L.fptr(depth), depth.shape[0]
        rec.code = L.fptr(c)
        rec.pose_is_obj_cam = 1 if pose_is_obj_cam else 0
        return rec

    @staticmethod
    def _result(o, code_len=64):
        """An out-record as the reference's result dict; ``code`` holds code_len values (the
        record's 64-wide code carries a 32-D code in its first 32, LocalMapping_util.cc:416-422)."""
        if o.is_good:
            return ForceKeyErrorDict(t_cam_obj=np.ctypeslib.as_array(o.t_cam_obj).reshape(4, 4).copy(),
                                     code=np.ctypeslib.as_array(o.code)[:code_len].copy(),
                                     is_good=True, loss=float(o.loss))
        return ForceKeyErrorDict(t_cam_obj=None, code=None, is_good=False, loss=float(o.loss))

    # ------------------------------------------------------------------ API
    def reconstruct_object(self, t_cam_obj, pts, rays, depth, code=None):
        """optimizer.py:90-205 (one object)."""
        return self.reconstruct_objects([(t_cam_obj, pts, rays, depth, code)])[0]

    def reconstruct_objects(self, objects, trace=False, pose_is_obj_cam=False):
        """Batched ``reconstruct_object``: ``objects`` is a list of
        ``(t_cam_obj, pts, rays, depth, code_or_None)``.  Returns a list of result dicts
        (and per-object traces when ``trace``)."""
        n = len(objects)
        if n == 0:
            return []
        keep = []
        ins = (L.ObjectIn * n)()
        for i, ob in enumerate(objects):
            t, p, r, d = ob[:4]
            c = ob[4] if len(ob) > 4 else None
            ins[i] = self._object_in(t, p, r, d, c, keep, pose_is_obj_cam)
        outs = (L.ObjectOut * n)()
        tr = None
        bufs = None
        if trace:
            it = max(1, self.num_iterations_joint_optim)
            bufs = [dict(H=np.zeros((it, 71, 71), np.float32), b=np.zeros((it, 71), np.float32),
                         dx=np.zeros((it, 71), np.float32), loss=np.zeros(it, np.float32),
                         sdf_loss=np.zeros(it, np.float32), render_loss=np.zeros(it, np.float32),
                         n_valid=np.zeros(it, np.int32), k=np.zeros(it, np.int32),
                         t_obj_cam=np.zeros((it, 4, 4), np.float32),
                         z=np.zeros((it, self.code_len), np.float32),
                         n_decoded=np.zeros(it, np.int32), n_refined=np.zeros(it, np.int32)) for _ in range(n)]
            tr = (L.Trace * n)()
            for i, bb in enumerate(bufs):
                tr[i] = L.Trace(*(L.fptr(bb[k]) for k in ("H", "b", "dx", "loss", "sdf_loss",
                                                          "render_loss")),
                                L.iptr(bb["n_valid"]), L.iptr(bb["k"]), L.fptr(bb["t_obj_cam"]),
                                L.fptr(bb["z"]), L.iptr(bb["n_decoded"]), L.iptr(bb["n_refined"]))
        t0 = time.time()
        ctx = self._ctx
        ctx.check(ctx.lib.dsr_reconstruct_batch(ctx.handle, self.decoder.handle,
                                                C.byref(self.params), n, ins, outs, tr),
                  "dsr_reconstruct_batch")
        if _VERBOSE:
            print("Reconstruction takes %f seconds" % (time.time() - t0))
        res = [self._result(outs[i], self.code_len) for i in range(n)]
        for i in range(n):
            res[i]["iters_done"] = int(outs[i].iters_done)
            res[i]["fail_reason"] = L.FAIL_REASONS.get(int(outs[i].fail_reason), "?")
        if trace:
            return res, bufs
        return res

    def reconstruct_objects_async(self, objects):
        """Start ``reconstruct_objects(objects)`` and return at once with a
        :class:`BatchHandle`: the inputs are uploaded (dsr_batch_create), the whole GN run is
        enqueued on the device (dsr_batch_run) and the host is free — e.g. for the
        LocalMapping thread's bundle adjustment, which the reference runs after the
        reconstructions (LocalMapping.cc:99-128) — until ``handle.wait()``."""
        return BatchHandle(self, objects)

    def reconstruct_keyframe_async(self, detections):
        """One keyframe's object reconstructions (LocalMapping_util.cc:165-206, 394-410) as
        ONE asynchronous batched call.  ``detections``: list of ``(t_cam_obj, pts, rays,
        depth, code, reconstructed)``.  For a detection whose object is not yet
        reconstructed the reference also runs the left-right flipped hypothesis —
        ``Sim3Two`` with columns 0 and 2 negated, i.e. ``t_cam_obj @ diag(-1, 1, -1, 1)``
        (exact in fp32) — and keeps it when the original's loss is larger
        (LocalMapping_util.cc:400-410; a failed run's loss takes part in that comparison as
        it does there).  Both hypotheses go into the same batch; ``wait()`` applies the
        choice and returns one result per detection."""
        return KeyframeHandle(self, detections)

    def reconstruct_keyframe(self, detections):
        return self.reconstruct_keyframe_async(detections).wait()

    MAX_SLOTS = 4
    # A slot batch is laid out for max_obj x max_rays x M ray samples whatever the fill, and every
    # run launches its render chunks over that capacity (~580 B of device memory per sample with
    # the kept ReLU masks).  A keyframe only uses a slot whose capacity is at most SLOT_WASTE x its
    # own ray count (or SLOT_MIN_RAYS), a slot only grows while it stays inside that bound, and no
    # slot exceeds SLOT_MAX_SAMPLES ray samples (2^24: ~9.7 GB); otherwise the keyframe runs as a
    # one-shot batch (INTEGRATION.md §2 states the bound)
    SLOT_WASTE = 4.0
    SLOT_MIN_RAYS = 8 * 1024
    SLOT_MAX_SAMPLES = 1 << 24

    def _slot_ok(self, n_obj, n_rays_cap, real_rays):
        cap = n_obj * n_rays_cap
        return (cap <= max(self.SLOT_WASTE * real_rays, self.SLOT_MIN_RAYS)
                and cap * self.num_depth_samples <= self.SLOT_MAX_SAMPLES)

    def _slot_for(self, objects):
        """A free fixed-capacity batch (dsr_batch_create_capacity) that holds ``objects``, or
        None (``keyframe_mode`` "oneshot", every slot busy with an in-flight keyframe, or no slot
        within the capacity bounds above: the keyframe then runs as a one-shot batch).  A free
        slot is grown (replaced by a larger one) only when the grown size stays inside the bounds;
        otherwise the keyframe gets a slot of its own — beside the others while fewer than
        MAX_SLOTS exist, else in place of the least recently used free slot (a small
        keyframe no longer destroys a large free slot and its captured graph)."""
        if self.keyframe_mode not in ("slot", "graph") or not objects:
            return None
        n = len(objects)
        rays = [_f32(ob[2], 3).shape[0] for ob in objects]
        need_p = max(_f32(ob[1], 3).shape[0] for ob in objects)
        need_r = max(rays)
        real = sum(rays)
        graph = self.keyframe_mode == "graph"
        self._slot_tick = getattr(self, "_slot_tick", 0) + 1
        free = [sl for sl in self._slots if not sl.busy and sl.graph == graph]
        for sl in free:
            if sl.fits(n, need_p, need_r) and self._slot_ok(sl.max_obj, sl.max_rays, real):
                sl.last_used = self._slot_tick
                return sl
        pad = lambda v: -(-v // 128) * 128  # noqa: E731
        cn, cp, cr = n, pad(need_p), pad(need_r)
        old = None
        for sl in free:                              # grow a free slot inside the bounds
            gn, gp, gr = max(cn, sl.max_obj), max(cp, sl.max_pts), max(cr, sl.max_rays)
            if self._slot_ok(gn, gr, real):
                old, (cn, cp, cr) = sl, (gn, gp, gr)
                break
        if old is None:
            if not self._slot_ok(cn, cr, real):
                return None
            if len(self._slots) >= self.MAX_SLOTS:   # evict the least recently used free slot
                if not free:
                    return None
                old = min(free, key=lambda sl: getattr(sl, "last_used", 0))
        if old is not None:
            self._slots.remove(old)
            old.close()
        sl = SlotBatch(self, cn, cp, cr, graph)
        sl.last_used = self._slot_tick
        self._slots.append(sl)
        return sl

    def close_slots(self):
        """Release the keyframe slot batches (their device memory goes back to the context pool)."""
        for sl in self._slots:
            sl.close()
        self._slots = []

    def estimate_pose_cam_obj(self, t_co_se3, scale, pts, code):
        """optimizer.py:46-87: pose-only SE(3) GN on the SDF term."""
        t = _f32(t_co_se3).reshape(4, 4)
        pts = _f32(pts, 3)
        c = _code(code, self.code_len)
        out = np.zeros((4, 4), np.float32)
        ctx = self._ctx
        ctx.check(ctx.lib.dsr_pose_only(ctx.handle, self.decoder.handle, C.byref(self.params),
                                        L.fptr(t), float(scale), L.fptr(pts), pts.shape[0],
                                        L.fptr(c), L.fptr(out)), "dsr_pose_only")
        return out

    def estimate_pose_cam_obj_batch(self, objects):
        """Batched ``estimate_pose_cam_obj``: ``objects`` is a list of
        ``(t_co_se3, scale, pts, code)``; every object's pose-only GN runs in one device
        pass per iteration (dsr_pose_only_batch).  The stereo path calls the single form
        once per associated object per keyframe (LocalMapping_util.cc:103-110)."""
        n = len(objects)
        if n == 0:
            return []
        keep = []
        ins = (L.PoseIn * n)()
        for i, (t, scale, pts, code) in enumerate(objects):
            t = _f32(t).reshape(4, 4)
            pts = _f32(pts, 3)
            c = _code(code, self.code_len)
            keep += [pts, c]
            rec = L.PoseIn()
            rec.t_co_se3[:] = t.reshape(-1).tolist()
            rec.scale = float(scale)
            rec.pts, rec.n_pts = L.fptr(pts), pts.shape[0]
            rec.code = L.fptr(c)
            ins[i] = rec
        out = np.zeros((n, 4, 4), np.float32)
        ctx = self._ctx
        ctx.check(ctx.lib.dsr_pose_only_batch(ctx.handle, self.decoder.handle, C.byref(self.params), n,
                                              ins, L.fptr(out)), "dsr_pose_only_batch")
        return [out[i] for i in range(n)]

    def reconstruct_objects_multi(self, objects, decoders, return_path=False):
        """``reconstruct_objects`` spread over several devices from ONE process
        (dsr_reconstruct_multi_ex): ``decoders`` holds one decoder handle per device (e.g.
        ``[decoder_from_state(state, specs, device=g) for g in range(n)]``); objects are
        LPT-partitioned, each device's shard runs on its own host thread and one RCCL gather
        returns the records to the first device (host memory when RCCL refuses the device
        list); ``return_path`` adds which ("rccl" / "host").  One process per GPU is
        reconstruct.parallel.reconstruct_sharded."""
        n = len(objects)
        if n == 0:
            return []
        keep = []
        ins = (L.ObjectIn * n)()
        for i, ob in enumerate(objects):
            ins[i] = self._object_in(*ob[:4], ob[4] if len(ob) > 4 else None, keep)
        outs = (L.ObjectOut * n)()
        nd = len(decoders)
        ctxs = (C.c_void_p * nd)(*[d.ctx.handle.value for d in decoders])
        decs = (C.c_void_p * nd)(*[d.handle.value for d in decoders])
        ctx = decoders[0].ctx
        path = C.c_int(-1)
        ctx.check(ctx.lib.dsr_reconstruct_multi_ex(ctxs, decs, nd, C.byref(self.params), n, ins, outs,
                                                   C.byref(path)), "dsr_reconstruct_multi_ex")
        res = [self._result(outs[i], self.code_len) for i in range(n)]
        for i in range(n):
            res[i]["iters_done"] = int(outs[i].iters_done)
            res[i]["fail_reason"] = L.FAIL_REASONS.get(int(outs[i].fail_reason), "?")
        if return_path:
            return res, ("rccl" if path.value == L.GATHER_RCCL else "host")
        return res

    def compute_sdf_loss_objectpoint_zhjd(self, pts_surface_obj, code):
        """optimizer.py:207-213: mean decoder SDF of object-frame points."""
        sdf = sdf_eval(self.decoder, _code(code, self.code_len), pts_surface_obj)
        mean_value = np.float32(np.mean(sdf)) if sdf.size else np.float32(np.nan)
        if _VERBOSE:
            print("[mapobject sdf loss]python:", mean_value)
        return float(mean_value)


class SlotBatch:
    """A fixed-capacity batch (dsr_batch_create_capacity) that keyframe after keyframe is
    refilled (dsr_batch_refill) and re-run — with ``graph``, as replays of ONE hipGraph."""

    def __init__(self, opt, max_obj, max_pts, max_rays, graph):
        self.opt = opt
        self.max_obj, self.max_pts, self.max_rays, self.graph = max_obj, max_pts, max_rays, graph
        self.busy = False
        ctx = opt._ctx
        h = C.c_void_p()
        ctx.check(ctx.lib.dsr_batch_create_capacity(ctx.handle, opt.decoder.handle, C.byref(opt.params), max_obj,
                                                    max_pts, max_rays, L.BATCH_GRAPH if graph else 0, C.byref(h)),
                  "dsr_batch_create_capacity")
        self.handle = h

    def fits(self, n, n_pts, n_rays):
        return n <= self.max_obj and n_pts <= self.max_pts and n_rays <= self.max_rays

    def close(self):
        h = getattr(self, "handle", None)
        if h is not None:
            try:
                self.opt._ctx.lib.dsr_batch_destroy(h)
            except Exception:
                pass
            self.handle = None

    def __del__(self):
        self.close()


class BatchHandle:
    """An in-flight batched reconstruction (Optimizer.reconstruct_objects_async); with a
    ``slot`` (SlotBatch) the objects are refilled into that fixed-capacity batch instead of a
    new batch being created."""

    def __init__(self, opt, objects, slot=None):
        self.opt = opt
        self.n = len(objects)
        self._h = None
        self._res = None
        self._slot = None
        if self.n == 0:
            self._res = []
            return
        keep = []
        ins = (L.ObjectIn * self.n)()
        for i, ob in enumerate(objects):
            ins[i] = opt._object_in(*ob[:4], ob[4] if len(ob) > 4 else None, keep)
        ctx = opt._ctx
        if slot is not None:
            ctx.check(ctx.lib.dsr_batch_refill(slot.handle, self.n, ins), "dsr_batch_refill")
            ctx.check(ctx.lib.dsr_batch_run(slot.handle), "dsr_batch_run")
            slot.busy = True
            self._slot = slot
            self._h = slot.handle
            return
        h = C.c_void_p()
        ctx.check(ctx.lib.dsr_batch_create(ctx.handle, opt.decoder.handle, C.byref(opt.params), self.n,
                                           ins, C.byref(h)), "dsr_batch_create")
        self._h = h
        # DSR_GRAPH=1: the whole GN run is captured as one hipGraph and replayed
        # (dsr_batch_graph is a no-op otherwise)
        ctx.check(ctx.lib.dsr_batch_graph(h), "dsr_batch_graph")
        ctx.check(ctx.lib.dsr_batch_run(h), "dsr_batch_run")

    def done(self) -> bool:
        """True once the device has finished (never blocks)."""
        if self._res is not None:
            return True
        ctx = self.opt._ctx
        rc = ctx.lib.dsr_batch_query(self._h)
        if rc < 0:
            ctx.check(rc, "dsr_batch_query")
        return rc == 1

    def wait(self):
        """Block until the run finishes; the list of result dicts, like reconstruct_objects."""
        if self._res is None:
            ctx = self.opt._ctx
            outs = (L.ObjectOut * self.n)()
            try:
                ctx.check(ctx.lib.dsr_batch_download(self._h, outs), "dsr_batch_download")
            finally:
                self._release()
            res = [Optimizer._result(outs[i], self.opt.code_len) for i in range(self.n)]
            for i in range(self.n):
                res[i]["iters_done"] = int(outs[i].iters_done)
                res[i]["fail_reason"] = L.FAIL_REASONS.get(int(outs[i].fail_reason), "?")
            self._res = res
        return self._res

    def _release(self):
        if self._slot is not None:           # the slot batch stays; its next fill may start
            self._slot.busy = False
            self._slot = None
        elif self._h is not None:
            self.opt._ctx.lib.dsr_batch_destroy(self._h)
        self._h = None

    def __del__(self):
        if getattr(self, "_h", None) is not None:
            try:
                if self._slot is not None:   # an abandoned keyframe: finish its run before reuse
                    self.opt._ctx.lib.dsr_batch_sync(self._h)
                self._release()
            except Exception:
                pass


FLIP = np.diag(np.array([-1.0, 1.0, -1.0, 1.0], np.float32))


class KeyframeHandle:
    """In-flight keyframe batch (Optimizer.reconstruct_keyframe_async)."""

    def __init__(self, opt, detections):
        objs, self.pairs = [], []
        for det in detections:
            t, pts, rays, depth = det[:4]
            code = det[4] if len(det) > 4 else None
            done = bool(det[5]) if len(det) > 5 else False
            i = len(objs)
            objs.append((t, pts, rays, depth, code))
            j = None
            if not done:
                j = len(objs)
                objs.append((np.asarray(t, np.float32).reshape(4, 4) @ FLIP, pts, rays, depth, code))
            self.pairs.append((i, j))
        self.batch = BatchHandle(opt, objs, opt._slot_for(objs))

    def done(self) -> bool:
        return self.batch.done()

    def wait(self):
        res = self.batch.wait()
        out = []
        for i, j in self.pairs:
            r = res[i]
            if j is not None and float(r["loss"]) > float(res[j]["loss"]):
                r = res[j]
            out.append(r)
        return out


def sdf_eval(decoder, code, pts, with_jac=False):
    """decode_sdf / get_batch_sdf_jacobian (loss_utils.py:51-113) on device."""
    ctx = decoder.ctx
    pts = _f32(pts, 3)
    c = _code(code, decoder.code_len)
    n = pts.shape[0]
    sdf = np.zeros(n, np.float32)
    jac = np.zeros((n, c.shape[0] + 3), np.float32) if with_jac else None
    ctx.check(ctx.lib.dsr_sdf_eval(ctx.handle, decoder.handle, L.fptr(c), L.fptr(pts), n,
                                   L.fptr(sdf), L.fptr(jac)), "dsr_sdf_eval")
    return (sdf, jac) if with_jac else sdf


class MeshExtractor(object):
    """optimizer.py:216-233 — grid decode + marching cubes on device (dsr_mesher_*).

    The voxel grid is reconstruct.utils.create_voxel_grid (bit-exact, including the
    reference's true-division shear) and is uploaded once, like the reference builds it
    once in __init__.  The reference meshes with skimage.measure.marching_cubes_lewiner
    (utils.py:119-140); the build's marching cubes (dsr_mc.hpp) is a closed,
    consistently oriented surface through the same level set — vertex/face ORDER and
    the triangulation of ambiguous cells are its own (parity unpinned: skimage is absent,
    DESIGN.md §3.5)."""

    def __init__(self, decoder, code_len=64, voxels_dim=64):
        self.decoder = decoder
        self.code_len = code_len
        self.voxels_dim = voxels_dim
        self.voxel_points = create_voxel_grid(vol_dim=self.voxels_dim)
        ctx = decoder.ctx
        h = C.c_void_p()
        ctx.check(ctx.lib.dsr_mesher_create(ctx.handle, decoder.handle, L.fptr(self.voxel_points),
                                            self.voxels_dim, C.byref(h)), "dsr_mesher_create")
        self._h = h
        d = self.voxels_dim
        self._verts = np.zeros((3 * d ** 3, 3), np.float32)
        self._faces = np.zeros((5 * (d - 1) ** 3, 3), np.int32)

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            try:
                self.decoder.ctx.lib.dsr_mesher_destroy(h)
            except Exception:
                pass
            self._h = None

    def decode_grid(self, code):
        """The (voxels_dim^3,) SDF grid of optimizer.py:226 (decode_sdf on device)."""
        return sdf_eval(self.decoder, _code(code, self.code_len), self.voxel_points)

    def extract_mesh_from_code(self, code, level=0.0):
        ctx = self.decoder.ctx
        c = _code(code, self.code_len)
        nv, nf = C.c_int(), C.c_int()
        ctx.check(ctx.lib.dsr_mesher_run(self._h, L.fptr(c), float(level), L.fptr(self._verts),
                                         self._verts.shape[0], L.iptr(self._faces), self._faces.shape[0],
                                         C.byref(nv), C.byref(nf)), "dsr_mesher_run")
        return ForceKeyErrorDict(vertices=self._verts[:nv.value].copy(), faces=self._faces[:nf.value].copy())

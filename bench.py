"""Benchmark: object-reconstructions/sec (2048 pts, 10 GN iters) on N MI355X.

One "step" = one full ``reconstruct_object`` (10 joint GN iterations, KITTI
parameters, configs/config_kitti.json:21-39) for every object of the job: by default
64 synthetic KITTI-like objects x 2048 surface points x (2048+200) rays (BASELINE.json
north star "2048 pts/object x 64 objects on 1 MI355X"), plus the device->host copy of
the results and, for N>1, one RCCL all-gather of the fixed-size result records
(SURVEY.md §8e).

Scaling: the job is FIXED (64 objects) and LPT-sharded across the N ranks
(reconstruct/parallel.py: ResidentShard) — strong scaling, the north star's
"≥6x strong scaling to 8 GPUs"; at N=1 this is exactly the metric's configuration.
``--weak`` instead gives every rank its own 64 objects.  ``--pts 4096`` is BASELINE
config 4 (64 objects x 4096 points, 8 per GPU at N=8).

Inputs are resident in HBM before the timed region (dsr_batch_create); each step
re-initialises the optimizer state on device and runs all iterations.  At N=1 rank 0
also reports: the exact-decode leg (``value_exact``: DSR_LITE=0, every ray sample
decoded in 3xFP16), the fp32-arithmetic leg (``fp32_leg``: the exact pass and the Jacobian
on the fp32-MFMA kernels, their rates against the 157.3 TF fp32 MFMA peak), the three MFMA
kernels' rooflines, the CPU baseline, the
Redwood keyframe leg (BASELINE config 5, ``keyframe``), one 16-object KITTI frame as one batch
(config 3 of the list, ``config2_frame``) and one object per ``reconstruct_object`` call
(``config1_single``).

Every N also runs a ``config4`` leg: BASELINE config 4 (64 objects x 4096 points, the same
LPT sharding, 8 per GPU at N=8), so one N=1,2,4,8 sweep gives both strong-scaling curves.

Usage: python bench.py [--gpus N --steps K --warmup W --objects B --pts P --weak]
       N>1: one process per GPU.  Under torch.distributed.run (WORLD_SIZE set) the ranks are
       the launcher's; without it bench.py starts ``torch.distributed.run --nproc-per-node N``
       itself as a child process (before any GPU call) and exits with its status.
"""
from __future__ import annotations

import argparse
import contextlib
import ctypes as C
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "dsp-slam-rgbd_amd"))
sys.path.insert(0, REPO)

import synthetic as S  # noqa: E402

FWD_MAC = 1_769_984     # algorithmic forward MACs / point (code broadcast folded), SURVEY §8
BWD_MAC = 1_835_520     # input-gradient backward MACs / point
FP16_MFMA_PEAK_TF = 2500.0          # dense fp16/bf16 MFMA, spec (MI355X_MICROARCH.md)
FP32_MFMA_PEAK_TF = 157.3           # dense fp32 MFMA, spec
FP16_MFMA_LOOP_TF = 1247.0          # the guide's bare 32x32x16 bf16 MFMA loop on random data (DVFS item 1)
SPLIT_PRODUCTS = 3                  # 3xFP16: hi*hi + hi*lo + lo*hi per fp32 product
DTYPE = ("fp16-mfma: 3xFP16 split (hi/lo fp16, fp32 accumulate) for every value that reaches "
         "an output + one-product fp16 classification of ray samples")

LAST_CREATE_S = None


def make_batch(dec, opt_params, n_obj, base_seed, n_pts=2048):
    """Resident batch of ``n_obj`` KITTI-like objects (seeds base_seed + i)."""
    from reconstruct import _libdsr as L

    keep, ins = [], (L.ObjectIn * n_obj)()
    for i in range(n_obj):
        o = S.kitti_object(i, base_seed=base_seed, n_pts=n_pts)
        arrs = [np.ascontiguousarray(a, np.float32) for a in (o.pts, o.rays, o.depth)]
        keep += arrs
        r = L.ObjectIn()
        r.t_cam_obj[:] = o.t_cam_obj.reshape(-1).tolist()
        r.pts, r.n_pts = L.fptr(arrs[0]), arrs[0].shape[0]
        r.rays, r.n_rays = L.fptr(arrs[1]), arrs[1].shape[0]
        r.depth, r.n_depth = L.fptr(arrs[2]), arrs[2].shape[0]
        r.code = None
        r.pose_is_obj_cam = 0
        ins[i] = r
    ctx = dec.ctx
    h = C.c_void_p()
    global LAST_CREATE_S
    t0 = time.perf_counter()
    ctx.check(ctx.lib.dsr_batch_create(ctx.handle, dec.handle, C.byref(opt_params), n_obj, ins,
                                       C.byref(h)), "dsr_batch_create")
    LAST_CREATE_S = time.perf_counter() - t0          # host -> HBM upload of the inputs (PCIe)
    return h, keep


def cpu_baseline(seconds_budget=30.0, n_pts=2048):
    """The CPU oracle (numpy, all host threads) on a bounded sample of the workload."""
    from deep_sdf.workspace import fold_state
    from oracle import dsr_oracle as O

    state = S.make_decoder(1234)
    dec = O.Decoder(fold_state(state, S.DEFAULT_SPECS))
    P = O.OptimParams.from_cfg(S.KITTI_OPTIM)
    o = S.kitti_object(0, n_pts=n_pts)
    t0 = time.time()
    # one metric-unit object, 10 GN iterations (stop early past the budget and extrapolate)
    n_fg = o.depth.shape[0]
    dobs = np.concatenate([o.depth, np.zeros(o.rays.shape[0] - n_fg)]).astype(np.float32)
    T = np.linalg.inv(o.t_cam_obj)
    z = np.zeros(64, np.float32)
    done = 0
    for _ in range(P.num_iterations):
        tr, Tn, zn = O.gn_step(dec, P, T, z, o.pts, o.rays, dobs, n_fg)
        done += 1
        if Tn is None:
            break
        T, z = Tn, zn
        if time.time() - t0 > seconds_budget:
            break
    dt = time.time() - t0
    per_obj = dt * P.num_iterations / done
    try:
        cores = len(os.sched_getaffinity(0))
    except Exception:
        cores = os.cpu_count()
    threads = int(os.environ.get("OMP_NUM_THREADS", cores))
    out = {"value": 1.0 / per_obj, "unit": "object-reconstructions/sec", "cores": min(threads, cores),
           "kind": "port",
           "sample": f"oracle/dsr_oracle.py (numpy fp32) on 1 KITTI object x {n_pts} pts, {done} of "
                     f"{P.num_iterations} GN iterations timed ({dt:.1f} s), extrapolated to 10"}
    out.update(reference_calibration(out["value"]))
    return out


def reference_calibration(port_value):
    """The port's speed relative to the reference's own CPU path, measured side by side in the
    build container (tools/cpu_calibrate.py -> profiles/r4_cpu_calibration.json: golden F4 kitti0,
    same thread counts, median of 3): reference-equivalent = port value / (port / reference).
    The box's host differs from that container; the ratio at the container's full thread count
    is the one applied."""
    path = os.path.join(REPO, "profiles", "r4_cpu_calibration.json")
    try:
        cal = json.load(open(path))
    except Exception:
        return {}
    th = cal["host"]["nproc"]
    ratio = cal["runs"].get(f"port_to_reference_ratio_{th}t")
    if not ratio:
        return {}
    return {"port_to_reference_ratio": round(ratio, 4), "reference_equivalent_value": port_value / ratio,
            "calibration": f"{os.path.relpath(path, REPO)}: port {cal['runs'][f'oracle_{th}t']['obj_per_s']:.4f} vs "
                           f"reference {cal['runs'][f'reference_{th}t']['obj_per_s']:.4f} obj/s at {th} threads "
                           f"(1 thread: ratio {cal['runs'].get('port_to_reference_ratio_1t', float('nan')):.3f})"}


def pmc_traffic(kernel):
    """HBM bytes per launch of `kernel` from the newest committed rocprofv3 PMC summary
    (profiles/<tag>_summary.json, written by tools/prof_summary.py from separate
    FETCH_SIZE / WRITE_SIZE passes over this same default workload), or None."""
    import glob

    best = None
    for f in sorted(glob.glob(os.path.join(REPO, "profiles", "*_summary.json"))):   # tag order
        try:
            d = json.load(open(f))
        except Exception:
            continue
        for name, e in d.get("pmc", {}).items():
            if kernel in name and "hbm_bytes_per_launch" in e:
                best = (e["hbm_bytes_per_launch"], os.path.relpath(f, REPO))
    return best


@contextlib.contextmanager
def env_set(**kv):
    """The bench legs' environment switches, restored on the way out even when a leg raises
    (a failed fp32 leg must not leave the later legs on the fp32 kernels)."""
    old = {k: os.environ.get(k) for k in kv}
    os.environ.update(kv)
    try:
        yield
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def stats_sum(acc, st):
    for k, _ in st._fields_:
        v = getattr(st, k)
        if k in ("lite_max_err",):
            acc[k] = max(acc.get(k, 0.0), v)
        elif k in ("lite_min_margin",):
            acc[k] = min(acc.get(k, 1e30), v)
        elif k in ("lite", "keep_masks", "surface_in_exact", "test_hooks", "lite_eligible", "audit",
                   "audit_shell", "audit_log2", "lite_margin0", "lite_floor", "lite_safety", "graph_captures",
                   "graph_replays", "n_groups", "graph_mode", "fwd_variant", "jac_variant", "lite_variant",
                   "split_ring"):
            acc[k] = v
        else:
            acc[k] = acc.get(k, 0) + v
    return acc


def kernel_rooflines(a):
    """Per-launch rate of the three MFMA kernels over the timed steps (HIP events on the
    stream each kernel runs on, dsr_batch_stats) against the spec peak and the guide's
    measured bare-MFMA-loop rate.  FLOPs are algorithmic and EXECUTED: the lite pass one
    fp16 product per MAC; the exact re-decode and the Jacobian fp32-equivalent (a 3xFP16
    MAC counts once, the spec peak is divided by 3); render points with kept ReLU masks
    run the backward chain only."""
    out = {}
    split_peak, split_loop = FP16_MFMA_PEAK_TF / SPLIT_PRODUCTS, FP16_MFMA_LOOP_TF / SPLIT_PRODUCTS
    ren_mac = BWD_MAC if a.get("keep_masks") else FWD_MAC + BWD_MAC
    # the fp32-MFMA kernels (DSR_FWD_VARIANT / DSR_JAC_VARIANT 0, the fp32 leg): fp32 products
    # against the fp32 MFMA peak (no bare-loop figure for them: the spec stands in)
    f32x, f32j = a.get("fwd_variant", 12) & 8 == 0, a.get("jac_variant", 12) & 8 == 0
    xname, xpeak, xloop, xnote = (("k_mlp_fwd (fp32 MFMA)", FP32_MFMA_PEAK_TF, FP32_MFMA_PEAK_TF, "fp32 products")
                                  if f32x else ("k_mlp_fwd16", split_peak, split_loop, "fp32-equivalent (3xFP16)"))

    def entry(name, flop, ms, launches, peak, loop, note):
        tf = flop / (ms * 1e-3) / 1e12 if ms > 0 else 0.0
        out[name] = {"achieved_tflops": round(tf, 2), "peak_tflops": round(peak, 1),
                     "frac_of_peak": round(tf / peak, 4), "guide_bf16_loop_tflops": round(loop, 1),
                     "frac_of_guide_loop": round(tf / loop, 4), "launches": launches,
                     "avg_launch_ms": round(ms / max(1, launches), 5),
                     "flop_per_launch": flop / max(1, launches), "flop_counted": note}

    if a.get("lite"):
        entry("k_mlp_fwd_lite_st", 2.0 * FWD_MAC * a["fwd_points"], a["fwd_ms"], a["fwd_launches"],
              FP16_MFMA_PEAK_TF, FP16_MFMA_LOOP_TF, "2*1,769,984 per decoded ray sample, fp16 products")
        surf = a["jac_surface_points"] if a.get("surface_in_exact") else 0
        entry(xname + " (exact pass: band + audit samples" + (", surface points)" if surf else ")"),
              2.0 * FWD_MAC * (a["refine_points"] + surf), a["refine_ms"], a["refine_launches"], xpeak,
              xloop, "2*1,769,984 per re-decoded sample" + (" and surface point" if surf else "") + ", " + xnote)
    else:
        entry(xname, 2.0 * FWD_MAC * a["fwd_points"], a["fwd_ms"], a["fwd_launches"],
              xpeak, xloop, "2*1,769,984 per decoded ray sample, " + xnote)
    if a.get("surface_in_exact"):      # every tile backward only (the exact pass ran the forwards)
        jflop = 2.0 * BWD_MAC * (a["jac_surface_points"] + a["jac_render_points"])
        note = "(N surface + K render points) x 2*1,835,520 (backward only, kept masks)"
    else:
        jflop = 2.0 * (FWD_MAC + BWD_MAC) * a["jac_surface_points"] + 2.0 * ren_mac * a["jac_render_points"]
        note = ("N surface points x 2*(1,769,984+1,835,520) + K render points x 2*"
                + ("1,835,520 (backward only, kept masks)" if a.get("keep_masks") else "(fwd+bwd)"))
    if f32j:
        entry("k_mlp_jac (fp32 MFMA)", jflop, a["jac_ms"], a["jac_launches"], FP32_MFMA_PEAK_TF, FP32_MFMA_PEAK_TF,
              note + ", fp32 products")
    else:
        entry("k_mlp_jac16", jflop, a["jac_ms"], a["jac_launches"], split_peak, split_loop, note)
    return out


def measured_mfma_loop(device=0, ms=300.0):
    """The device's bare v_mfma_f32_16x16x32_f16 loop on random register operands, every
    SIMD busy (csrc/dsr_diag.hip): the fp16 MFMA rate the chip sustains under load on this
    box (it lowers its clock under MFMA load, MI355X_MICROARCH.md 'DVFS give-back'), for
    one and two waves per SIMD (the decoder kernels run two).  None if unavailable."""
    path = os.path.join(REPO, "dsp-slam-rgbd_amd", "csrc", "libdsr_diag.so")
    if not os.path.exists(path):
        return None
    lib = C.CDLL(path)
    out = {}
    for w in (1, 2):
        tf, t = C.c_float(), C.c_float()
        if lib.dsr_diag_mfma_f16(device, w, 0, C.c_float(ms), C.byref(tf), C.byref(t)) != 0:
            return None
        out[f"waves_per_simd_{w}"] = round(tf.value, 1)
    out["tflops"] = max(out.values())
    out["note"] = ("bare fp16 MFMA loop (16x16x32, 8 accumulators, random operands in registers, "
                   "every SIMD busy), measured after the timed region on the same device")
    return out


def keyframe_leg(dec, n_keyframes=12, objects=4):
    """BASELINE config 5: Redwood parameters, per keyframe `objects` new detections, each
    also run as its flipped hypothesis (LocalMapping_util.cc:394-410), 512 points, 5 GN
    iterations — one batched asynchronous call per keyframe
    (Optimizer.reconstruct_keyframe_async), so the host is free for the reference's
    LocalBundleAdjustment (LocalMapping.cc:99-128) while the GPU works.  Reports ms per
    keyframe (uploads and download included) and the host time spent while batches were in
    flight, for each keyframe mode: "graph" (the default: one fixed-capacity slot batch refilled
    per keyframe, every run a replay of ONE captured hipGraph), "slot" (the same slot run
    eagerly) and "oneshot" (a new batch per keyframe)."""
    from reconstruct.optimizer import Optimizer
    from reconstruct.utils import ForceKeyErrorDict

    kfs = []
    for k in range(n_keyframes):
        dets = []
        for i in range(objects):
            o = S.redwood_object(100 * k + i)
            dets.append((o.t_cam_obj, o.pts, o.rays, o.depth, None, False))
        kfs.append(dets)
    modes = {}
    for mode in ("oneshot", "slot", "graph"):
        opt = Optimizer(dec, ForceKeyErrorDict(data_type="Redwood", optimizer=S.REDWOOD_OPTIM))
        opt.keyframe_mode = mode
        opt.reconstruct_keyframe(kfs[0])              # warm-up (and, for "graph", the capture)
        t0 = time.perf_counter()
        host_s = 0.0
        good = 0
        for dets in kfs:
            h = opt.reconstruct_keyframe_async(dets)
            t1 = time.perf_counter()
            while not h.done():                       # stand-in for host-side BA
                pass
            host_s += time.perf_counter() - t1
            good += sum(r["is_good"] for r in h.wait())
        dt = time.perf_counter() - t0
        modes[mode] = {"ms_per_keyframe": round(dt / n_keyframes * 1e3, 3),
                       "host_free_ms_per_keyframe": round(host_s / n_keyframes * 1e3, 3), "good_detections": good}
        if mode != "oneshot":
            from reconstruct import _libdsr as L

            st = L.Stats()
            opt._ctx.check(opt._ctx.lib.dsr_batch_stats(opt._slots[0].handle, C.byref(st)), "stats")
            modes[mode].update(slot_batches=len(opt._slots), graph_captures=st.graph_captures,
                               graph_replays=st.graph_replays)
        opt.close_slots()
    out = {"keyframes": n_keyframes, "detections_per_keyframe": objects, "objects_per_keyframe_batch": 2 * objects,
           "mode": "graph", "modes": modes,
           "note": "Redwood params, 512 pts, 712 rays, 5 iters; original + flipped hypothesis per detection in one "
                   "async batch (includes H2D upload and result download)"}
    out.update(modes["graph"])
    return out


def device_record(device, torch):
    """This rank's HIP device: index, PCI location and name (ranks.devices in the line)."""
    rec = {"rank": int(os.environ.get("RANK", "0")), "host": socket.gethostname(), "hip_device": int(device),
           "pci_bus_id": None, "pci_domain_id": None, "name": None}
    try:
        p = torch.cuda.get_device_properties(int(device))
        rec.update(pci_bus_id=int(p.pci_bus_id), pci_domain_id=int(p.pci_domain_id), name=p.name)
    except Exception:
        pass
    return rec


def spawn_ranks(n):
    """``--gpus n`` without a launcher: run this script under torch.distributed.run with n
    local ranks (RCCL rendezvous on 127.0.0.1) as a CHILD process — this process never
    touches the GPU — and return its exit status."""
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def fp32_algorithmic(a, steps, elapsed, stats_steps=None):
    """SURVEY.md §8(d)'s algorithmic count: per object and iteration 2*1,769,984*(N + N_valid)
    + 2*1,835,520*(N + K) FLOP (fp32 decoder, every in-ball sample decoded, Jacobian points
    re-forwarded), summed over the timed steps, against the fp32 MFMA peak.  It exceeds that
    peak because the build decodes fewer samples (exact early ray termination), classifies most
    of them with one fp16 product and runs the rest as 3xFP16 — the fractions below."""
    n, nv, k = a.get("jac_surface_points", 0), a.get("inball_points", 0), a.get("jac_render_points", 0)
    flop = (2.0 * FWD_MAC * (n + nv) + 2.0 * BWD_MAC * (n + k)) * steps / (stats_steps or steps)
    tf = flop / elapsed / 1e12 if elapsed > 0 else 0.0
    dec = a.get("fwd_points", 0)
    return {"flop_per_step": flop / max(1, steps), "achieved_tflops": round(tf, 1),
            "fp32_mfma_peak_tflops": FP32_MFMA_PEAK_TF, "frac_of_fp32_peak": round(tf / FP32_MFMA_PEAK_TF, 3),
            "decoded_fraction_of_inball": round(dec / max(1, nv), 4),
            "one_product_fraction_of_decoded": round(1.0 - a.get("refine_points", 0) / max(1, dec), 4)
            if a.get("lite") else 0.0,
            "note": "SURVEY §8(d) count over the timed steps / their time; > 1 of the fp32 peak because "
                    "early ray termination skips samples and the lite pass classifies most decoded samples "
                    "with one fp16 product (DESIGN.md §3.3-3.4)"}


def record_rows(res):
    """Gathered out-records as float32 rows (loss, is_good, iters, T[16], code[64]) — what
    --dump-records writes, for bitwise comparisons across rank counts."""
    return np.array([[r["loss"], float(r["is_good"]), r["iters_done"]]
                     + (list(np.asarray(r["t_cam_obj"]).reshape(-1)) + list(r["code"])
                        if r["is_good"] else [np.nan] * 80) for r in res], np.float32)


def config4_leg(opt, rank, coll_dev, barrier, dist, torch, steps=3, n_obj=64, n_pts=4096, dump=""):
    """BASELINE config 4: ONE job of 64 synthetic KITTI objects x 4096 points, LPT-sharded over
    the ranks (8 per GPU at N=8) with the record gather; same timing rules as the main line."""
    from reconstruct.parallel import ResidentShard

    objs = []
    for i in range(n_obj):
        o = S.kitti_object(i, base_seed=3000, n_pts=n_pts)
        objs.append((o.t_cam_obj, o.pts, o.rays, o.depth, None))
    shard = ResidentShard(opt, objs, device=coll_dev)
    try:
        shard.run()                                   # warm-up
        barrier()
        t0 = time.perf_counter()
        good = 0
        res = None
        for _ in range(steps):
            res = shard.run()
            if res is not None:
                good += sum(int(r["is_good"]) for r in res)
        barrier()
        el = time.perf_counter() - t0
        if dump and res is not None:
            np.save(dump, record_rows(res))
        if dist is not None:
            t = torch.tensor([el], dtype=torch.float64, device=coll_dev or "cpu")
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el = float(t.item())
        return {"value": n_obj * steps / el, "unit": "object-reconstructions/sec", "steps": steps,
                "ms_per_step": el / steps * 1e3, "objects": n_obj, "pts": n_pts, "rays": n_pts + 200,
                "shard_objects": [len(s) for s in shard.shards], "good_fraction": good / float(n_obj * steps),
                "note": f"BASELINE configs[3]: {n_obj} x {n_pts}-point objects, one job LPT-sharded over the ranks"}
    finally:
        shard.close()


def small_legs(opt, objs, steps=3):
    """BASELINE configs[2] and configs[1] taken literally, beside the 64-object metric job:
    one KITTI frame of 16 objects x 2048 pts as one resident batch (obj/s), and ONE object per
    call through the reference's own entry point, ``Optimizer.reconstruct_object``
    (LocalMapping_util.cc:181-194 calls it once per detection): ms per call, uploads and
    download included."""
    import torch
    from reconstruct.parallel import ResidentShard

    sh = ResidentShard(opt, objs[:16])
    try:
        sh.run()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            sh.run()
        dt = time.perf_counter() - t0
    finally:
        sh.close()
    o = objs[0]
    opt.reconstruct_object(*o[:4])                      # warm-up (pooled buffers, events)
    t1 = time.perf_counter()
    for _ in range(5):
        r = opt.reconstruct_object(*o[:4])
    single = (time.perf_counter() - t1) / 5
    return {"config2_frame": {"objects": 16, "value": 16 * steps / dt, "unit": "object-reconstructions/sec",
                              "ms_per_frame": dt / steps * 1e3,
                              "note": "BASELINE configs[2]: one KITTI frame of 16 x 2048-pt objects, one batch"},
            "config1_single": {"ms_per_call": single * 1e3, "is_good": bool(r.is_good),
                               "note": "BASELINE configs[1]: one 2048-pt object, 10 GN iters, per "
                                       "Optimizer.reconstruct_object call (H2D + run + D2H)"}}


def parse_args():
    """Arguments and world size.  ``--gpus N`` (N > 1) without a launcher: spawn the ranks and
    exit with their status; under a launcher without ``--gpus``: the launcher's rank count."""
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--objects", type=int, default=64, help="objects in the job (per GPU with --weak)")
    ap.add_argument("--pts", type=int, default=2048, help="surface points per object (config 4: 4096)")
    ap.add_argument("--weak", action="store_true", help="every rank its own --objects objects")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extra", action="store_true", help="skip the exact-decode and keyframe legs")
    ap.add_argument("--no-config4", action="store_true", help="skip the 64 x 4096-point config-4 leg")
    ap.add_argument("--dump-records", default="", help="rank 0 writes the last step's gathered records (.npy; "
                                                       "the config-4 leg's to <name>_c4.npy)")
    ap.add_argument("--c4-objects", type=int, default=64, help="config-4 leg: objects (rehearsals only)")
    ap.add_argument("--c4-pts", type=int, default=4096, help="config-4 leg: points per object (rehearsals only)")
    gpus_given = any(a == "--gpus" or a.startswith("--gpus=") for a in sys.argv[1:])
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if not gpus_given:                       # under a launcher without --gpus: its ranks
        args.gpus = world
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world} ranks were launched")
    return args, world


def main():
    args, world = parse_args()
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    # DSR_BENCH_BACKEND=gloo (host tensors) rehearses the N>1 code path with several ranks on
    # one device, which RCCL refuses; the driver's runs use RCCL ("nccl") over xGMI
    backend = os.environ.get("DSR_BENCH_BACKEND", "nccl")
    import torch

    # DSR_BENCH_FORCE_DIST=1: initialise the process group even for one rank, so a one-GPU box
    # runs the N>1 code path (RCCL collectives on device tensors) end to end
    if world > 1 or os.environ.get("DSR_BENCH_FORCE_DIST") == "1":
        import torch.distributed as dist
        from reconstruct.parallel import rank_device

        # rank r binds device r; under RCCL a node with fewer visible devices than ranks exits
        # non-zero here instead of running its ranks on device 0 (parallel.rank_device)
        local = rank_device(local, int(os.environ.get("LOCAL_WORLD_SIZE", world)), backend,
                            torch.cuda.device_count())
        if backend == "nccl":
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    coll_dev = torch.device("cuda", local) if backend == "nccl" and dist is not None else None
    os.environ["DSR_DEVICE"] = str(local)        # Context.get() default: this rank's device

    from deep_sdf.workspace import decoder_from_state
    from reconstruct import _libdsr as L
    from reconstruct.optimizer import Optimizer
    from reconstruct.parallel import ResidentShard
    from reconstruct.utils import ForceKeyErrorDict

    state = S.make_decoder(1234)
    dec = decoder_from_state(state, S.DEFAULT_SPECS, device=local)
    opt = Optimizer(dec, ForceKeyErrorDict(data_type="KITTI", optimizer=S.KITTI_OPTIM))
    n_job = args.objects * (world if args.weak else 1)
    objs = []
    for i in range(n_job):
        o = S.kitti_object(i, base_seed=1000, n_pts=args.pts)
        objs.append((o.t_cam_obj, o.pts, o.rays, o.depth, None))
    t0 = time.perf_counter()
    shard = ResidentShard(opt, objs, device=coll_dev)
    create_s = time.perf_counter() - t0
    lib, ctx = dec.ctx.lib, dec.ctx

    def barrier():
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    for _ in range(args.warmup):
        shard.run()

    barrier()
    acc = {}
    n_good = 0
    gather_s = 0.0
    t0 = time.perf_counter()
    # per-step kernel statistics (HIP-event times of every decoder launch, counters): read after
    # every step at N = 1, where they feed the roofline; with several ranks only after the
    # timed region, for the last step (~200 event queries + 3 copies per read, ~0.3 ms: 1% of
    # an 8-object shard's step, which the strong-scaling value would otherwise carry)
    per_step_stats = world == 1
    for _ in range(args.steps):
        res = shard.run()
        gather_s += shard.last_gather_s
        if shard.handle is not None and per_step_stats:
            st = L.Stats()
            ctx.check(lib.dsr_batch_stats(shard.handle, C.byref(st)), "stats")
            stats_sum(acc, st)
        if res is not None:
            n_good += sum(int(r["is_good"]) for r in res)
    barrier()
    elapsed = time.perf_counter() - t0
    stats_steps = args.steps
    if shard.handle is not None and not per_step_stats:
        st = L.Stats()
        ctx.check(lib.dsr_batch_stats(shard.handle, C.byref(st)), "stats")
        stats_sum(acc, st)
        stats_steps = 1
    per_rank = [elapsed]
    ranks = {"world_size": world, "shard_objects": [len(s) for s in shard.shards],
             "gather_ms_per_step": round(gather_s / args.steps * 1e3, 4)}
    me = device_record(dec.ctx.device, torch)
    ranks["devices"] = [me]
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device=coll_dev or "cpu")
        all_t = [torch.zeros_like(t) for _ in range(world)]
        dist.all_gather(all_t, t)
        per_rank = [float(x.item()) for x in all_t]
        elapsed = max(per_rank)
        devs = [None] * world
        dist.all_gather_object(devs, me)
        ranks.update(backend=dist.get_backend(), world_size_observed=dist.get_world_size(),
                     rank_seconds=[round(x, 4) for x in per_rank], devices=devs,
                     distinct_devices=len({(d["host"], d["pci_bus_id"], d["pci_domain_id"]) for d in devs}))
    if args.dump_records and rank == 0 and res is not None:
        np.save(args.dump_records, record_rows(res))
    value = n_job * args.steps / elapsed
    roof = kernel_rooflines(acc) if acc else {}
    loop = measured_mfma_loop(local) if rank == 0 and acc and not args.no_extra else None
    if loop:
        for name, e in roof.items():     # the split kernels' fp32-equivalent rate is 1/3 of fp16
            k = 1.0 if "lite" in name else 1.0 / SPLIT_PRODUCTS
            e["measured_loop_tflops"] = round(loop["tflops"] * k, 1)
            e["frac_of_measured_loop"] = round(e["achieved_tflops"] / (loop["tflops"] * k), 4)
    if rank == 0:
        dom = "k_mlp_fwd_lite_st" if acc.get("lite") else "k_mlp_fwd16"
        r = roof.get(dom, {})
        out = {
            "metric": f"object-reconstructions/sec ({args.pts} pts, 10 GN iters)",
            "value": value,
            "value_basis": "inputs resident in HBM before the timed region (dsr_batch_create); "
                           "host_inclusive_value adds the PCIe upload (SURVEY §8(d) end-to-end)",
            "unit": "object-reconstructions/sec",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak" if args.weak else "strong",
            "vs_baseline": None,
            "dtype": DTYPE,
            "data": "synthetic (seeded DeepSDF 8x512 decoder + KITTI-like objects, SURVEY.md §8d)",
            "config": {"workload": f"{n_job} objects x {args.pts} pts x ({args.pts}+200) rays x 50 depth "
                                   "samples, 10 GN iters, KITTI params (BASELINE configs[1] unit; "
                                   + ("64 objects per GPU)" if args.weak else
                                      f"one {n_job}-object job LPT-sharded over {world} GPU(s))"),
                       "objects": n_job, "objects_on_rank0": len(shard.mine), "pts": args.pts,
                       "rays": args.pts + 200, "iters": 10,
                       "parallelism": f"object-sharded x{world}" + (" (weak)" if args.weak else " (strong)")},
            "roofline": {"bound": "mfma", "kernel": dom,
                         "achieved": r.get("achieved_tflops"), "peak": r.get("peak_tflops"),
                         "unit": "TFLOP/s", "frac": r.get("frac_of_peak"),
                         "traffic": None, "traffic_unit": "bytes/launch (HBM+MALL, PMC)",
                         "avg_launch_ms": r.get("avg_launch_ms"), "launches": r.get("launches"),
                         "flop_per_launch": r.get("flop_per_launch")},
            "rooflines": roof,
            "mfma_loop": loop,
            "early_ray_termination": {"samples_decoded": acc.get("fwd_points"),
                                      "samples_in_ball": acc.get("inball_points"),
                                      "decoded_fraction": round(acc.get("fwd_points", 0)
                                                                / max(1, acc.get("inball_points", 1)), 4)},
            "lite_pass": None if not acc.get("lite") else {
                "refine_points": acc["refine_points"], "audit_points": acc["audit_points"],
                "refine_fraction": round(acc["refine_points"] / max(1, acc["fwd_points"]), 4),
                "audit_fraction": round(acc["audit_points"] / max(1, acc["fwd_points"]), 4),
                "audit_violations": acc["lite_audit_violations"],
                "redo_objects": acc["lite_redo_objects"],
                "max_observed_lite_error": acc["lite_max_err"], "min_margin": acc["lite_min_margin"]},
            "jac_points": {"surface": acc.get("jac_surface_points"), "render": acc.get("jac_render_points"),
                           "render_backward_only": bool(acc.get("keep_masks"))},
            "fp32_algorithmic": fp32_algorithmic(acc, args.steps, elapsed, stats_steps) if acc else None,
            "lite_broken_blocks": acc.get("lite_broken_blocks"),
            "test_hooks": acc.get("test_hooks"),
            # the lite pass's guard as the timed batches ran it (dsr_stats, ABI 8) and the decoder's
            # load-time qualification (dsr_decoder_info): not switchable without DSR_TEST_HOOKS=1
            "lite_guard": {"decoder_lite_eligible": bool(acc.get("lite_eligible")), "audit": acc.get("audit"),
                           "audit_shell_margins": acc.get("audit_shell"), "audit_hashed_share_log2": acc.get("audit_log2"),
                           "margin_first_iteration": acc.get("lite_margin0"), "margin_floor": acc.get("lite_floor"),
                           "margin_safety": acc.get("lite_safety"),
                           "decoder_probe": {k: dec.info[k] for k in ("lite_probe_ratio", "lite_probe_max_err",
                                                                     "lite_probe_max_err_all", "probe_points",
                                                                     "probe_codes", "probe_ms")}},
            "ranks": ranks,
            # device wall of one run (HIP events around dsr_batch_run's work, rank 0): the rest of
            # ms_per_step is host time (launch, download, packing, stats)
            "device_ms_per_step": round(acc["total_ms"] / stats_steps, 3) if acc else None,
            "stats_steps": stats_steps,
            "good_fraction": n_good / float(n_job * args.steps),
            # inputs handed over in host memory: the upload added to one step (set below from a
            # batch created against the context's warm pool — the steady state of a stream of jobs;
            # the first creation in a process also pays its hipMallocs / event creation)
            "host_inclusive_value": None,
            "host_inclusive_value_cold": n_job / (elapsed / args.steps + create_s),
            "batch_create_ms_cold": create_s * 1e3,
            "cpu_baseline": None,
        }
        tr = pmc_traffic(dom)
        if tr is not None:
            out["roofline"]["traffic"] = tr[0]
            out["roofline"]["traffic_source"] = tr[1]
    shard.close()
    t0 = time.perf_counter()
    warm = ResidentShard(opt, objs, device=coll_dev)   # the same job again, from the pooled blocks
    create_warm_s = time.perf_counter() - t0
    warm.close()
    if rank == 0:
        out["batch_create_ms"] = create_warm_s * 1e3
        out["host_inclusive_value"] = n_job / (elapsed / args.steps + create_warm_s)
    if not args.no_config4 and not args.weak:
        c4 = config4_leg(opt, rank, coll_dev, barrier, dist, torch, steps=min(args.steps, 3), n_obj=args.c4_objects,
                         n_pts=args.c4_pts,
                         dump=args.dump_records[:-4] + "_c4.npy" if args.dump_records.endswith(".npy") else "")
        if rank == 0:
            out["config4"] = c4
    if world == 1 and not args.no_extra:
        # exact-decode leg: DSR_LITE=0 (every in-ball sample decoded in 3xFP16), same job
        k = min(args.steps, 3)
        with env_set(DSR_LITE="0"):
            ex = ResidentShard(opt, objs)
            ex.run()
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            for _ in range(k):
                ex.run()
            dt = time.perf_counter() - t1
            ex.close()
        out["value_exact"] = n_job * k / dt
        out["value_exact_note"] = "DSR_LITE=0: no classification pass, every in-ball sample decoded exactly"
        # fp32-arithmetic leg: the same job with the exact pass and the
        # Jacobian on the fp32-MFMA kernels (test hooks DSR_FWD_VARIANT / DSR_JAC_VARIANT 0; the
        # lite classification stays fp16): what fp32 arithmetic costs, and those kernels' rate
        # against the 157.3 TF fp32 MFMA peak
        with env_set(DSR_TEST_HOOKS="1", DSR_FWD_VARIANT="0", DSR_JAC_VARIANT="0"):
            f32 = ResidentShard(opt, objs)
            try:
                f32.run()
                torch.cuda.synchronize()
                t1 = time.perf_counter()
                for _ in range(k):
                    f32.run()
                dt = time.perf_counter() - t1
                st32 = L.Stats()
                ctx.check(lib.dsr_batch_stats(f32.handle, C.byref(st32)), "stats")
            finally:
                f32.close()
        a32 = stats_sum({}, st32)
        out["fp32_leg"] = {"value": n_job * k / dt, "unit": "objects/s",
                           "fwd_variant": a32.get("fwd_variant"), "jac_variant": a32.get("jac_variant"),
                           "rooflines": {name: {k2: e[k2] for k2 in ("achieved_tflops", "peak_tflops", "frac_of_peak",
                                                                     "avg_launch_ms", "launches")}
                                         for name, e in kernel_rooflines(a32).items()},
                           "note": "exact pass + Jacobian on v_mfma_f32_16x16x4_f32 (fp32 products), lite "
                                   "classification unchanged; kernel rates over the last run's launches"}
        # the three MFMA kernels with the job on ONE stream: per-launch rates without the other
        # object group's concurrent kernels inside each launch's duration; the
        # headline roofline above is the timed region's, with both groups overlapping
        with env_set(DSR_STREAMS="1"):
            one = ResidentShard(opt, objs)
            try:
                one.run()
                one.run()
                st1 = L.Stats()
                ctx.check(lib.dsr_batch_stats(one.handle, C.byref(st1)), "stats")
            finally:
                one.close()
        r1 = kernel_rooflines(stats_sum({}, st1))
        out["rooflines_one_stream"] = {name: {k2: e[k2] for k2 in ("achieved_tflops", "peak_tflops", "frac_of_peak",
                                                                   "avg_launch_ms", "launches")}
                                       for name, e in r1.items()}
        out["keyframe"] = keyframe_leg(dec)
        out.update(small_legs(opt, objs))
    if rank == 0:
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(n_pts=args.pts)
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

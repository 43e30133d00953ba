"""Benchmark: object-reconstructions/sec (2048 pts, 10 GN iters) on N MI355X.

One "step" = one full ``reconstruct_object`` (10 joint GN iterations, KITTI
parameters, configs/config_kitti.json:21-39) for every object of this rank's
batch: 64 synthetic KITTI-like objects x 2048 surface points x (2048+200) rays
per GPU (BASELINE.json north-star "2048 pts/object x 64 objects on 1 MI355X"),
plus the device->host copy of the results and, for N>1, one RCCL all-gather of
the fixed-size result records.  Objects are independent, so the
batch is sharded across ranks with no data-path collective: weak scaling.

Inputs are resident in HBM before the timed region (dsr_batch_create); each
step re-initialises the optimizer state on device and runs all iterations.

Usage: python bench.py [--gpus N --steps K --warmup W --objects B]
       (N>1 through torch.distributed.run, one process per GPU)
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "dsp-slam-rgbd_amd"))
sys.path.insert(0, REPO)

import synthetic as S  # noqa: E402

FWD_MAC = 1_769_984     # algorithmic forward MACs / point (code broadcast folded), SURVEY §8
BWD_MAC = 1_835_520     # input-gradient backward MACs / point
FP32_MFMA_PEAK_TF = 157.3
FP16_MFMA_PEAK_TF = 2500.0          # dense fp16/bf16 MFMA (MI355X_MICROARCH.md)
SPLIT_PRODUCTS = 3                  # 3xFP16: hi*hi + hi*lo + lo*hi per fp32 product


LAST_CREATE_S = None


def make_batch(dec, opt_params, n_obj, base_seed):
    from reconstruct import _libdsr as L

    keep, ins = [], (L.ObjectIn * n_obj)()
    for i in range(n_obj):
        o = S.kitti_object(i, base_seed=base_seed)
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


def cpu_baseline(seconds_budget=30.0):
    """The CPU oracle (numpy, all host threads) on a bounded sample of the workload."""
    from deep_sdf.workspace import fold_state
    from oracle import dsr_oracle as O

    state = S.make_decoder(1234)
    dec = O.Decoder(fold_state(state, S.DEFAULT_SPECS))
    P = O.OptimParams.from_cfg(S.KITTI_OPTIM)
    o = S.kitti_object(0)
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
    return {"value": 1.0 / per_obj, "unit": "object-reconstructions/sec", "cores": min(threads, cores),
            "kind": "port",
            "sample": f"oracle/dsr_oracle.py (numpy fp32) on 1 KITTI object x 2048 pts, {done} of "
                      f"{P.num_iterations} GN iterations timed ({dt:.1f} s), extrapolated to 10"}


def pmc_traffic(kernel="k_mlp_fwd16"):
    """HBM bytes per launch of `kernel` from the newest committed rocprofv3 PMC summary
    (profiles/<tag>_summary.json, written by tools/prof_summary.py from separate
    FETCH_SIZE / WRITE_SIZE passes over this same default workload), or None."""
    import glob

    best = None
    for f in sorted(glob.glob(os.path.join(REPO, "profiles", "*_summary.json"))):   # tag order r1 < r1b < ...
        try:
            d = json.load(open(f))
        except Exception:
            continue
        for name, e in d.get("pmc", {}).items():
            if kernel in name and "hbm_bytes_per_launch" in e:
                best = (e["hbm_bytes_per_launch"], os.path.relpath(f, REPO))
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--objects", type=int, default=64, help="objects per GPU")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    # DSR_BENCH_BACKEND=gloo (host tensors) rehearses the N>1 code path with several ranks on
    # one device, which RCCL refuses; the driver's runs use RCCL ("nccl") over xGMI
    backend = os.environ.get("DSR_BENCH_BACKEND", "nccl")
    if world > 1:
        import torch
        import torch.distributed as dist

        if backend == "nccl":
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
            local = local % max(1, torch.cuda.device_count())
    coll_dev = "cuda" if backend == "nccl" else "cpu"

    from deep_sdf.workspace import decoder_from_state
    from reconstruct import _libdsr as L

    state = S.make_decoder(1234)
    dec = decoder_from_state(state, S.DEFAULT_SPECS, device=local)
    params = L.optim_params(S.KITTI_OPTIM)
    n_obj = args.objects
    batch, keep = make_batch(dec, params, n_obj, base_seed=1000 + rank * 100000)
    lib, ctx = dec.ctx.lib, dec.ctx
    outs = (L.ObjectOut * n_obj)()
    rec = np.zeros((n_obj, 96), np.float32)

    def step():
        ctx.check(lib.dsr_batch_run(batch), "dsr_batch_run")
        ctx.check(lib.dsr_batch_download(batch, outs), "dsr_batch_download")
        for i in range(n_obj):
            o = outs[i]
            rec[i, :16] = o.t_cam_obj
            rec[i, 16:80] = o.code
            rec[i, 80] = o.loss
            rec[i, 81] = o.is_good
        if dist is not None:
            import torch

            t = torch.from_numpy(rec).to(coll_dev)
            gath = torch.empty((world * n_obj, 96), dtype=torch.float32, device=t.device)
            dist.all_gather_into_tensor(gath, t)       # RCCL over xGMI
            torch.cuda.synchronize()

    for _ in range(args.warmup):
        step()
    if dist is not None:
        import torch

        dist.barrier()
        torch.cuda.synchronize()
    ctx.check(lib.dsr_batch_sync(batch), "sync")
    t0 = time.perf_counter()
    fwd_ms = jac_ms = 0.0
    fwd_pts = jac_pts = inball_pts = fwd_launches = 0
    refine_ms, refine_pts, lite_err, lite_margin, lite = 0.0, 0, 0.0, 1e30, False
    n_good = 0
    for _ in range(args.steps):
        step()
        st = L.Stats()
        ctx.check(lib.dsr_batch_stats(batch, C.byref(st)), "stats")
        fwd_ms += st.fwd_ms
        jac_ms += st.jac_ms
        fwd_pts += st.fwd_points
        jac_pts += st.jac_points
        inball_pts += st.inball_points
        fwd_launches += st.fwd_launches
        refine_ms += st.refine_ms
        refine_pts += st.refine_points
        lite_err = max(lite_err, st.lite_max_err)
        lite_margin = min(lite_margin, st.lite_min_margin)
        lite = bool(st.lite)
        n_good += sum(int(outs[i].is_good) for i in range(n_obj))
    ctx.check(lib.dsr_batch_sync(batch), "sync")
    if dist is not None:
        import torch

        torch.cuda.synchronize()
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        import torch

        t = torch.tensor([elapsed], dtype=torch.float64, device=coll_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    total_obj = n_obj * world * args.steps
    value = total_obj / elapsed
    fwd_flop = 2.0 * FWD_MAC * fwd_pts
    jac_flop = 2.0 * (FWD_MAC + BWD_MAC) * jac_pts
    fwd_tf = fwd_flop / (fwd_ms * 1e-3) / 1e12 if fwd_ms > 0 else 0.0
    job_tf = (fwd_flop + jac_flop) / elapsed / 1e12
    variant = int(os.environ.get("DSR_FWD_VARIANT", "12"))
    if variant & 8:
        split_peak = FP16_MFMA_PEAK_TF / SPLIT_PRODUCTS
        split_note = ("fp32-equivalent peak of the 3xFP16 split: 2.5 PF dense fp16 MFMA / 3 products; "
                      "achieved counts algorithmic fp32 FLOPs (executed fp16 MFMA FLOPs = 3x)")
    else:
        split_peak = FP32_MFMA_PEAK_TF
        split_note = "fp32 MFMA dense peak"
    if lite:
        kernel, kname = ("k_mlp_fwd_lite_st",
                         "k_mlp_fwd_lite_st (one-product fp16 classification pass over ray samples)")
        peak_tf, peak_note = FP16_MFMA_PEAK_TF, "dense fp16 MFMA peak (one product per MAC, fp32 accumulate)"
    else:
        kernel, kname = "k_mlp_fwd16", "k_mlp_fwd16 (decode_sdf on ray samples, 3xFP16)"
        peak_tf, peak_note = split_peak, split_note
    refine_flop = 2.0 * FWD_MAC * refine_pts
    refine_tf = refine_flop / (refine_ms * 1e-3) / 1e12 if refine_ms > 0 else 0.0
    if rank == 0:
        out = {
            "metric": "object-reconstructions/sec (2048 pts, 10 GN iters)",
            "value": value,
            "unit": "object-reconstructions/sec",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "mfma_precision": ("ray samples classified by a one-product fp16 pass; every value that "
                               "reaches an output (band samples, Jacobian points) decoded in 3xFP16 split "
                               "(hi/lo fp16, fp32 accumulate; fp32-class, parity suite green)") if lite else
                              ("3xFP16 split (hi/lo fp16 pieces, power-of-2 scaled, fp32 accumulate; "
                               "fp32-class accuracy, parity suite green)") if variant & 8 else "fp32 MFMA",
            "data": "synthetic (seeded DeepSDF 8x512 decoder + KITTI-like objects, SURVEY.md §8d)",
            "config": {"workload": f"{n_obj} objects/GPU x 2048 pts x (2048+200) rays x 50 depth "
                                   "samples, 10 GN iters, KITTI params (BASELINE configs[1] unit, "
                                   "batched as north-star 64 objects/GPU)",
                       "objects_per_gpu": n_obj, "pts": 2048, "rays": 2248, "iters": 10,
                       "parallelism": f"object-sharded x{world}"},
            "roofline": {"bound": "mfma", "kernel": kname,
                         "achieved": round(fwd_tf, 3), "peak": round(peak_tf, 1),
                         "unit": "TFLOP/s", "frac": round(fwd_tf / peak_tf, 4),
                         "peak_note": peak_note,
                         "traffic": None, "traffic_unit": "bytes/launch (HBM+MALL, PMC)",
                         "launches": fwd_launches,
                         "flop_per_launch": fwd_flop / max(1, fwd_launches),
                         "avg_launch_ms": fwd_ms / max(1, fwd_launches)},
            "early_ray_termination": {"samples_decoded": fwd_pts, "samples_in_ball": inball_pts,
                                      "decoded_fraction": round(fwd_pts / max(1, inball_pts), 4)},
            "lite_pass": None if not lite else {
                "refine_points": refine_pts, "refine_fraction": round(refine_pts / max(1, fwd_pts), 4),
                "refine_kernel": "k_mlp_fwd16 (3xFP16)", "refine_ms_per_step": refine_ms / args.steps,
                "refine_tflops": round(refine_tf, 3), "refine_peak": round(split_peak, 1),
                "max_observed_lite_error": lite_err, "min_margin": lite_margin},
            "job_tflops": round(job_tf, 3),
            "jac_kernel_tflops": round(jac_flop / (jac_ms * 1e-3) / 1e12, 3) if jac_ms > 0 else 0.0,
            "good_fraction": n_good / float(n_obj * args.steps),
            # inputs handed over in host memory: dsr_batch_create's upload added to one step
            "host_inclusive_value": n_obj * world / (elapsed / args.steps + LAST_CREATE_S),
            "batch_create_ms": LAST_CREATE_S * 1e3,
            "cpu_baseline": None,
        }
        tr = pmc_traffic(kernel)
        if tr is not None:
            out["roofline"]["traffic"] = tr[0]
            out["roofline"]["traffic_source"] = tr[1]
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline()
        print(json.dumps(out), flush=True)
    lib.dsr_batch_destroy(batch)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

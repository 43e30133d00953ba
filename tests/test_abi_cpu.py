"""The C ABI (include/dsr.h) without a GPU: the library loads, exports every declared
entry point, its struct layouts match the ctypes mirror, and it fails loudly (no
silent fallback) when no gfx950 device is present."""
from __future__ import annotations

import os
import re
import subprocess
import tempfile

import pytest

from conftest import REPO

HDR = os.path.join(REPO, "include", "dsr.h")


def declared_functions():
    txt = open(HDR).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\*?\s+\**(dsr_\w+)\s*\(", txt, flags=re.M)))


def test_header_declares_expected_entry_points():
    fns = declared_functions()
    for f in ("dsr_ctx_create", "dsr_decoder_load", "dsr_reconstruct_batch", "dsr_sdf_eval",
              "dsr_pose_only", "dsr_batch_run"):
        assert f in fns


def test_library_exports_every_declared_symbol():
    from reconstruct import _libdsr as L

    lib = L.load_library()
    fns = declared_functions()
    assert set(fns) == set(L.SIGNATURES), set(fns) ^ set(L.SIGNATURES)
    for f in fns:
        assert hasattr(lib, f), f
    out = subprocess.run(["nm", "-D", "--defined-only", L.lib_path()], capture_output=True,
                         text=True, check=True).stdout
    for f in fns:
        assert re.search(rf"\bT {f}$", out, flags=re.M), f
    assert lib.dsr_abi_version() == L.ABI_VERSION


def test_diag_library_exports_the_mfma_loop():
    """libdsr_diag.so (bench.py's measured MFMA ceiling) is built beside libdsr.so."""
    path = os.path.join(REPO, "dsp-slam-rgbd_amd", "csrc", "libdsr_diag.so")
    out = subprocess.run(["nm", "-D", "--defined-only", path], capture_output=True, text=True,
                         check=True).stdout
    assert re.search(r"\bT dsr_diag_mfma_f16$", out, flags=re.M)


STRUCTS = {"dsr_decoder_desc": "DecoderDesc", "dsr_optim_params": "OptimParams",
           "dsr_object_in": "ObjectIn", "dsr_object_out": "ObjectOut", "dsr_trace": "Trace",
           "dsr_stats": "Stats", "dsr_pose_in": "PoseIn", "dsr_decoder_info": "DecoderInfo"}


def test_struct_layouts_match_ctypes():
    import ctypes

    from reconstruct import _libdsr as L

    lines = ['#include <stdio.h>', '#include <stddef.h>', f'#include "{HDR}"', "int main(void){"]
    for cname, pyname in STRUCTS.items():
        lines.append(f'printf("{pyname} size %zu\\n", sizeof({cname}));')
        for fld, _ in getattr(L, pyname)._fields_:
            lines.append(f'printf("{pyname} {fld} %zu\\n", offsetof({cname}, {fld}));')
    lines.append("return 0;}")
    with tempfile.TemporaryDirectory() as d:
        src = os.path.join(d, "layout.c")
        exe = os.path.join(d, "layout")
        open(src, "w").write("\n".join(lines))
        subprocess.run(["gcc", "-std=c99", "-o", exe, src], check=True)
        out = subprocess.run([exe], capture_output=True, text=True, check=True).stdout
    for line in out.strip().splitlines():
        py, what, val = line.split()
        cls = getattr(L, py)
        if what == "size":
            assert ctypes.sizeof(cls) == int(val), line
        else:
            assert getattr(cls, what).offset == int(val), line


def test_no_device_fails_loudly():
    """Without a visible gfx950 GPU, creating a context raises (no CPU fallback)."""
    from reconstruct import _libdsr as L

    try:
        import torch
        if torch.cuda.is_available():
            pytest.skip("a GPU is visible")
    except ImportError:
        pass
    with pytest.raises(L.DsrError):
        L.Context(0)


def test_missing_library_fails_loudly(tmp_path):
    from reconstruct import _libdsr as L

    with pytest.raises(L.DsrError):
        L.load_library(str(tmp_path / "nope.so"))


def test_c_caller_links_and_fails_loudly_without_a_device():
    """examples/dsr_c_smoke.c — the ABI from C, no Python: it links
    against libdsr.so, its DSR_ABI_VERSION matches the library's, and without a HIP device
    context creation reports -3 (no CPU fallback)."""
    exe = os.path.join(REPO, "dsp-slam-rgbd_amd", "csrc", "dsr_c_smoke")
    assert os.path.isfile(exe), "built by make -C dsp-slam-rgbd_amd/csrc"
    p = subprocess.run([exe], capture_output=True, text=True, timeout=60)
    assert p.returncode == 0, p.stderr
    rc = int(p.stdout.split()[-1])
    assert rc in (0, -3)


@pytest.mark.parametrize("exe_name", ["dsr_c_stress", "dsr_c_stress_asan"])
def test_c_stress_no_device_paths(exe_name):
    """examples/dsr_c_stress.c without inputs: the argument checks and error reporting of
    the entry points that validate before touching the device, against the shipped library
    and against libdsr_asan.so (host code under AddressSanitizer + UBSan, leak checking
    on).  The device paths of the same driver run in test_gpu_api.py."""
    exe = os.path.join(REPO, "dsp-slam-rgbd_amd", "csrc", exe_name)
    if exe_name.endswith("_asan") and not os.path.isfile(exe):
        pytest.skip("host-sanitized build absent (make -C dsp-slam-rgbd_amd/csrc check)")
    assert os.path.isfile(exe), "built by make -C dsp-slam-rgbd_amd/csrc"
    p = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stdout + p.stderr
    assert "stress ok" in p.stdout


def test_gather_layout_of_the_multi_device_entry_point():
    """dsr_reconstruct_multi_ex gathers every device's shard of fixed-size
    dsr_object_out records to device 0 in one ncclGather of equal slots: object i is record
    dev[i] * maxn + slot[i].  dsr_gather_layout (host-only, no device) is that layout: the LPT
    partition of reconstruct/parallel.py (cost n_rays * M + n_pts), input order within a shard,
    every record position used once, maxn the largest shard."""
    import ctypes

    import numpy as np

    from reconstruct import _libdsr as L
    from reconstruct.parallel import lpt_partition

    lib = L.load_library()
    rng = np.random.default_rng(5)
    for n_obj, n_dev in ((1, 1), (7, 2), (64, 8), (13, 8), (5, 8)):
        ins = (L.ObjectIn * n_obj)()
        costs = []
        for i in range(n_obj):
            ins[i].n_rays = int(rng.integers(0, 3000))
            ins[i].n_pts = int(rng.integers(0, 4096))
            costs.append(ins[i].n_rays * 50 + ins[i].n_pts)
        dev = np.zeros(n_obj, np.int32)
        slot = np.zeros(n_obj, np.int32)
        maxn = ctypes.c_int(0)
        assert lib.dsr_gather_layout(n_obj, ins, 50, n_dev, L.iptr(dev), L.iptr(slot), ctypes.byref(maxn)) == 0
        shards = lpt_partition(costs, n_dev)
        for g in range(n_dev):
            mine = sorted(np.nonzero(dev == g)[0].tolist())
            assert mine == sorted(shards[g]), (n_obj, n_dev, g)
            assert slot[mine].tolist() == list(range(len(mine)))       # input order within the shard
        assert maxn.value == max(len(s) for s in shards)
        pos = dev.astype(np.int64) * maxn.value + slot
        assert len(set(pos.tolist())) == n_obj and pos.max() < n_dev * maxn.value
    assert ctypes.sizeof(L.ObjectOut) % 4 == 0                          # records gathered as bytes

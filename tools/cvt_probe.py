"""The activation split's conversions on the GPU (diagnostic): hi = v_cvt_pk_f16_f32(x), lo =
v_fma_mixlo/hi_f16(-hi + x) exactly as dsr_mlp16.hpp: write_split, against round-to-nearest-even
(numpy) — rounding mode, fp16 denormal handling, and the mean of hi + lo - x."""
import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
lib = ctypes.CDLL(os.path.join(HERE, "libmfma_numerics.so"))
rng = np.random.default_rng(3)
n = 1 << 20
for name, x in [("x in [2^-6, 2^14), positive (scaled activations)", np.exp2(rng.uniform(-6, 14, n)).astype(np.float32)),
                ("x tiny positive (lo in fp16 denormals)", np.exp2(rng.uniform(-16, -4, n)).astype(np.float32)),
                ("x normal, both signs", (rng.standard_normal(n) * 100).astype(np.float32))]:
    h = np.zeros(n, np.float16)
    lo = np.zeros(n, np.float16)
    assert lib.cvt(ctypes.c_void_p(x.ctypes.data), ctypes.c_void_p(h.ctypes.data), ctypes.c_void_p(lo.ctypes.data), n) == 0
    h_rne = x.astype(np.float16)
    l_rne = (x - h_rne.astype(np.float32)).astype(np.float16)
    l_fromgpu_h = (x - h.astype(np.float32)).astype(np.float16)
    err = h.astype(np.float64) + lo.astype(np.float64) - x.astype(np.float64)
    rel = err / np.abs(x.astype(np.float64))
    print(f"{name}: hi != RNE {np.mean(h != h_rne):.4f}, lo != RNE(x - hi) {np.mean(lo != l_fromgpu_h):.4f} "
          f"(lo == 0 where RNE is not: {np.mean((lo == 0) & (l_fromgpu_h != 0)):.4f}); mean (hi+lo-x)/|x| {rel.mean():+.3e} "
          f"rms {np.sqrt((rel ** 2).mean()):.3e}; numpy split mean {((h_rne.astype(np.float64) + l_rne - x) / np.abs(x)).mean():+.3e}",
          flush=True)

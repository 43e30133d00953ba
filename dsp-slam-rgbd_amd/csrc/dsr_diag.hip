// dsr_diag.hip — measurement helper, not part of the product path (libdsr_diag.so).
//
// The practical fp16 MFMA ceiling of THIS device: a bare loop of
// v_mfma_f32_16x16x32_f16 (the instruction every libdsr decoder kernel issues) on random
// register operands, every SIMD busy, no memory traffic.  Under load the MI355X lowers its
// clock (MI355X_MICROARCH.md "DVFS give-back"), so the spec's 2.5 PF dense fp16 peak is
// not what an MFMA-bound kernel can reach; bench.py reports each decoder kernel's rate
// against both this measured loop and the spec peak.
#include <hip/hip_runtime.h>

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float floatx4 __attribute__((ext_vector_type(4)));

namespace {

__device__ __forceinline__ _Float16 rnd_half(unsigned x, int zero) {
  x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
  // uniform in [-1/64, 1/64): products stay small, accumulators finite over the loop
  return zero ? (_Float16)0.f : (_Float16)(((float)(x >> 8) * (1.f / 16777216.f) - 0.5f) * (1.f / 32.f));
}

template <int NACC>
__global__ __launch_bounds__(256) void k_mfma_loop(int iters, int zero, float* out) {
  const unsigned gid = blockIdx.x * blockDim.x + threadIdx.x;
  half8 a[4], b[4];                    // 4 operand pairs in turn: the MFMA inputs toggle
  for (int k = 0; k < 4; ++k)
    for (int i = 0; i < 8; ++i) {
      a[k][i] = rnd_half(gid * 64 + 16 * k + i, zero);
      b[k][i] = rnd_half(gid * 64 + 16 * k + 8 + i + 0x9e3779b9u, zero);
    }
  floatx4 acc[NACC];
  for (int j = 0; j < NACC; ++j) acc[j] = floatx4{0.f, 0.f, 0.f, 0.f};
  for (int it = 0; it < iters; ++it) {        // iters x 16 rounds of NACC MFMAs
#pragma unroll
    for (int u = 0; u < 16; ++u)
#pragma unroll
      for (int j = 0; j < NACC; ++j)
        acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[(j + u) & 3], b[(j + u + 1) & 3], acc[j], 0, 0, 0);
  }
  float s = 0.f;
  for (int j = 0; j < NACC; ++j) s += acc[j][0] + acc[j][1] + acc[j][2] + acc[j][3];
  out[gid] = s;
}

}  // namespace

extern "C" {

// Runs the loop for about `target_ms` (after one warm-up launch of the same length) with
// `waves_per_simd` waves on every SIMD (1 or 2); zero != 0 feeds all-zero operands.
// Returns 0 and the achieved dense TFLOP/s (2 x 16 x 16 x 32 per MFMA) and wall ms.
int dsr_diag_mfma_f16(int device, int waves_per_simd, int zero, float target_ms, float* tflops, float* ms) {
  if (!tflops || !ms || waves_per_simd < 1 || waves_per_simd > 2) return -2;
  if (hipSetDevice(device) != hipSuccess) return -1;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) != hipSuccess) return -1;
  const int blocks = prop.multiProcessorCount * waves_per_simd;     // 4 waves per block = 1 per SIMD
  float* out = nullptr;
  if (hipMalloc(&out, sizeof(float) * blocks * 256) != hipSuccess) return -1;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  constexpr int NACC = 8;
  int iters = 256;
  float t = 0.f;
  int rc = 0;
  for (int pass = 0; pass < 3; ++pass) {       // calibrate, warm up at the target length, measure
    hipEventRecord(e0, nullptr);
    hipLaunchKernelGGL(k_mfma_loop<NACC>, dim3(blocks), dim3(256), 0, nullptr, iters, zero, out);
    hipEventRecord(e1, nullptr);
    if (hipEventSynchronize(e1) != hipSuccess) { rc = -1; break; }
    hipEventElapsedTime(&t, e0, e1);
    if (pass == 0 && t > 0.f) iters = (int)(iters * (target_ms / t)) + 1;
  }
  if (rc == 0) {
    const double flop = 2.0 * 16 * 16 * 32 * NACC * 16.0 * iters * blocks * 4;
    *tflops = (float)(flop / (t * 1e-3) / 1e12);
    *ms = t;
  }
  hipEventDestroy(e0);
  hipEventDestroy(e1);
  hipFree(out);
  return rc;
}

}  // extern "C"

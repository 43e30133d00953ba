// dsr_proto.hip — timing prototype (NOT the product): the "VGPR-resident activations" division of a
// CU for the lite decoder pass, measured instead of costed.
//
// Structure: one wave per SIMD (4 waves, 256 threads per workgroup, one workgroup per CU), 32 points
// per wave (128 per CU, as the shipped lite kernel's tile).  A layer's output Y[512 x 32] = W[512 x 512]
// . X[512 x 32] runs on v_mfma_f32_32x32x16_f16: X is the B operand and stays in registers (32 k steps x
// 8 halves = 128 VGPRs: the previous layer's accumulators converted in place — a 32x32 accumulator's
// registers 8s..8s+7 ARE k step s of the next product's B fragment once the weight columns are permuted
// at load time, cdna_hip_programming.md §3), the 16 accumulators (512 rows) take 256 registers, and the
// weights stream L2 -> LDS by LDS-DMA (global_load_lds_dwordx4, four 1 KiB pieces per wave per k step)
// through a ring of NS 16 KiB slabs shared by the 4 waves, one raw barrier per k step.  Per layer: 32 k
// steps x 16 MFMAs, one ds_read_b128 A fragment per MFMA; epilogue = scale + ReLU + fp16 convert into the
// B registers.  No tile I/O, no classification, random operands: an UPPER bound of what the structure can
// do, for the kill criterion (>= +8 % over the shipped lite kernel's one-stream rate).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <utility>
#include <vector>

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float floatx16 __attribute__((ext_vector_type(16)));

namespace {
constexpr int NS = 4;                 // LDS ring slabs
constexpr int SLAB = 16 * 1024;       // one 16-deep k step of all 512 rows: 16 row blocks x 1 KiB
constexpr int LAYERS = 7;             // lin1..lin7
constexpr int KSTEPS = 32;            // 512 / 16

// piece rb of global k step g: (layer, k step) = ((g / 32) % 7, g % 32); 64 lanes x 16 B, A-fragment order
__device__ __forceinline__ void issue(const _Float16* __restrict__ W, char* lds, int g, int w, int lane) {
  const int layer = (g >> 5) % LAYERS, ks = g & 31;
  const _Float16* src = W + ((size_t)((layer * KSTEPS + ks) * 16) * 64 + lane) * 8;
  char* dst = lds + (g % NS) * SLAB;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int rb = w + 4 * i;
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(src + (size_t)rb * 512),
                                     (__attribute__((address_space(3))) void*)(dst + rb * 1024), 16, 0, 0);
  }
}
}  // namespace

// ds_read_b128 by inline asm: hipcc's own waits for compiler-issued LDS reads were lgkmcnt(0) in this
// kernel (never counted), so the reads are issued here and waited for by the counted, fragment-tied
// s_waitcnt above (`after` orders the read behind the MFMA that frees its ring slot)
template <int OFF>
__device__ __forceinline__ half8 lds_read(unsigned base, const floatx16& after) {
  half8 v;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v) : "v"(base), "n"(OFF), "a"(after));
  return v;
}

__global__ __launch_bounds__(256) void k_proto_vres(const _Float16* __restrict__ W, int n_tiles, float* __restrict__ out) {
  __shared__ __attribute__((aligned(1024))) char lds[NS * SLAB];
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  half8 b[KSTEPS];
  floatx16 acc[16];
  float sum = 0.f;
  int g = 0;
  // slabs 0 .. NS-2 in flight; step g waits for slab g+1 (one step AHEAD of its use), so the first A
  // fragments of the next step can be read during this one: a ring of RING fragments per wave
  constexpr int RING = 4;
#pragma unroll
  for (int i = 0; i < NS - 1; ++i) issue(W, lds, i, w, lane);
  asm volatile("s_waitcnt vmcnt(4)" ::: "memory");      // slab 0 (own pieces)
  __builtin_amdgcn_s_barrier();
  half8 ar[RING];
  const unsigned base = (unsigned)(uintptr_t)(__attribute__((address_space(3))) char*)lds + lane * 16;
  [&]<int... I>(std::integer_sequence<int, I...>) { ((ar[I] = lds_read<I * 1024>(base, acc[0])), ...); }(
      std::make_integer_sequence<int, RING>{});
  for (int tile = blockIdx.x; tile < n_tiles; tile += gridDim.x) {
#pragma unroll
    for (int t = 0; t < KSTEPS; ++t)
#pragma unroll
      for (int j = 0; j < 8; ++j)
        b[t][j] = (_Float16)((float)(((tile * 131 + t * 7 + j * 3 + lane * 5) & 255) - 128) * (1.f / 256.f));
#pragma unroll 1
    for (int layer = 0; layer < LAYERS; ++layer) {
#pragma unroll
      for (int rb = 0; rb < 16; ++rb) acc[rb] = floatx16{};
      auto kstep = [&]<int T>(std::integral_constant<int, T>) {
        // own pieces of slab g+1 landed (the 4 youngest glds are slab g+2's); after the barrier every
        // wave's slab g+1 is complete and every wave is past its reads of slab g-1 (consumed by step
        // g-1's MFMAs), which slab g+NS-1 then overwrites
        asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        issue(W, lds, g + NS - 1, w, lane);
        [&]<int... R>(std::integer_sequence<int, R...>) {
          ([&] {
            constexpr int rb = R, rn = rb + RING;
            constexpr int off = rn < 16 ? (T % NS) * SLAB + rn * 1024 : ((T + 1) % NS) * SLAB + (rn - 16) * 1024;
            // counted wait tied to the fragment: reads rb+1..rb+3 may still be in flight
            asm volatile("s_waitcnt lgkmcnt(3)" : "+v"(ar[rb % RING]));
            acc[rb] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ar[rb % RING], b[T], acc[rb], 0, 0, 0);
            ar[rb % RING] = lds_read<off>(base, acc[rb]);
          }(), ...);
        }(std::make_integer_sequence<int, 16>{});
        ++g;
      };
      [&]<int... T>(std::integer_sequence<int, T...>) { (kstep(std::integral_constant<int, T>{}), ...); }(
          std::make_integer_sequence<int, KSTEPS>{});
      // epilogue: registers 8s..8s+7 of row block rb -> k step 2 rb + s of the next layer's B
#pragma unroll
      for (int rb = 0; rb < 16; ++rb)
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          half8 v;
#pragma unroll
          for (int j = 0; j < 8; ++j) v[j] = (_Float16)fmaxf(acc[rb][8 * s2 + j] * 0.0625f, 0.f);
          b[2 * rb + s2] = v;
        }
    }
#pragma unroll
    for (int t = 0; t < KSTEPS; ++t) sum += (float)b[t][0] + (float)b[t][7];
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  out[blockIdx.x * blockDim.x + threadIdx.x] = sum;
}

extern "C" {

// Runs the prototype on `device` for `reps` launches of `tiles` 128-point tiles and reports the fp16
// product rate (7 x 512 x 512 x 128 x 2 FLOP per tile) and the average launch time (HIP events).
int dsr_proto_vres(int device, int tiles, int reps, float* tflops, float* ms_per_launch, float* checksum) {
  if (hipSetDevice(device) != hipSuccess) return -1;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) != hipSuccess) return -1;
  const size_t nw = (size_t)LAYERS * KSTEPS * 16 * 64 * 8;
  std::vector<_Float16> hw(nw);
  uint32_t s = 12345u;
  for (auto& x : hw) {
    s = s * 1664525u + 1013904223u;
    x = (_Float16)(((float)(s >> 8) / 16777216.f - 0.5f) * 0.25f);
  }
  _Float16* dw = nullptr;
  float* dout = nullptr;
  const int grid = prop.multiProcessorCount;
  if (hipMalloc(&dw, nw * sizeof(_Float16)) != hipSuccess) return -1;
  if (hipMalloc(&dout, sizeof(float) * grid * 256) != hipSuccess) { hipFree(dw); return -1; }
  hipMemcpy(dw, hw.data(), nw * sizeof(_Float16), hipMemcpyHostToDevice);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipLaunchKernelGGL(k_proto_vres, dim3(grid), dim3(256), 0, 0, (const _Float16*)dw, tiles, dout);   // warm-up
  hipEventRecord(e0, 0);
  for (int r = 0; r < reps; ++r)
    hipLaunchKernelGGL(k_proto_vres, dim3(grid), dim3(256), 0, 0, (const _Float16*)dw, tiles, dout);
  hipEventRecord(e1, 0);
  const hipError_t err = hipEventSynchronize(e1);
  float ms = 0.f;
  hipEventElapsedTime(&ms, e0, e1);
  std::vector<float> ho((size_t)grid * 256);
  hipMemcpy(ho.data(), dout, sizeof(float) * ho.size(), hipMemcpyDeviceToHost);
  double cs = 0.0;
  for (float v : ho) cs += v;
  hipEventDestroy(e0);
  hipEventDestroy(e1);
  hipFree(dw);
  hipFree(dout);
  if (err != hipSuccess || hipGetLastError() != hipSuccess) return -2;
  const double flop = (double)LAYERS * 512.0 * 512.0 * 128.0 * 2.0 * tiles * reps;
  *ms_per_launch = ms / reps;
  *tflops = (float)(flop / (ms * 1e-3) / 1e12);
  *checksum = (float)cs;
  return 0;
}

}  // extern "C"

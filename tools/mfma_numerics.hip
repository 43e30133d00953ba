// MFMA rounding probe (diagnostic, not product code): one wave per trial computes
//   D = mfma_f32_16x16x32_f16(A, B, C)      (mode 0)
//   D = mfma(A1, B1, mfma(A0, B0, C))        (mode 1: two chained k steps, 64-deep)
//   D = mfma_f32_16x16x4_f32(A, B, C)        (mode 2)
// with the gfx950 operand layouts (lane l: A[row l&15][k = 8(l>>4) + j], B[k][col l&15];
// D[row 4(l>>4) + r][col l&15]; f32 16x16x4: k = l>>4).  tools/mfma_numerics.py compares D
// with the exact sums rounded to nearest-even and toward zero.
#include <hip/hip_runtime.h>

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float floatx4 __attribute__((ext_vector_type(4)));

__global__ void k_probe(const _Float16* A, const _Float16* B, const float* C, float* D, int mode) {
  const int t = blockIdx.x, l = threadIdx.x;
  const int row = l & 15, kg = l >> 4;
  floatx4 c;
  for (int r = 0; r < 4; ++r) c[r] = C[t * 256 + (4 * kg + r) * 16 + row];
  if (mode == 2) {
    const float* Af = reinterpret_cast<const float*>(A) + t * 64;
    const float* Bf = reinterpret_cast<const float*>(B) + t * 64;
    c = __builtin_amdgcn_mfma_f32_16x16x4f32(Af[row * 4 + kg], Bf[kg * 16 + row], c, 0, 0, 0);
  } else {
    const int nk = mode == 1 ? 2 : 1;
    for (int s = 0; s < nk; ++s) {
      half8 a, b;
      for (int j = 0; j < 8; ++j) {
        a[j] = A[(size_t)t * 16 * 32 * nk + row * 32 * nk + 32 * s + 8 * kg + j];
        b[j] = B[(size_t)t * 32 * nk * 16 + (32 * s + 8 * kg + j) * 16 + row];
      }
      c = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
    }
  }
  for (int r = 0; r < 4; ++r) D[t * 256 + (4 * kg + r) * 16 + row] = c[r];
}

// one split-fp16 GEMM output block the way dsr_mlp16.hpp: gemm16_ring chains it: 16 k steps of
// 32, each al.bh, ah.bl, ah.bh into the running accumulator (K = 512); A [t][2][16][512],
// B [t][2][512][16] (piece 0 hi, 1 lo), D [t][16][16]
// mode 0: one chain (al.bh, ah.bl, ah.bh onto the running sum: the shipped kernels); 1: each k
// step's three products from zero, then a VALU add; 2: the lo corrections from zero, the hi
// product onto the running sum, then a VALU add of the corrections
__global__ void k_split_chain(const _Float16* A, const _Float16* B, float* D, int mode) {
  const int t = blockIdx.x, l = threadIdx.x, row = l & 15, kg = l >> 4;
  const _Float16* Ah = A + (size_t)t * 2 * 16 * 512;
  const _Float16* Al = Ah + 16 * 512;
  const _Float16* Bh = B + (size_t)t * 2 * 512 * 16;
  const _Float16* Bl = Bh + 512 * 16;
  floatx4 c = {0.f, 0.f, 0.f, 0.f};
  for (int s = 0; s < 16; ++s) {
    half8 ah, al, bh, bl;
    for (int j = 0; j < 8; ++j) {
      const int k = 32 * s + 8 * kg + j;
      ah[j] = Ah[row * 512 + k]; al[j] = Al[row * 512 + k];
      bh[j] = Bh[k * 16 + row]; bl[j] = Bl[k * 16 + row];
    }
    const floatx4 z = {0.f, 0.f, 0.f, 0.f};
    if (mode == 0) {
      c = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, bh, c, 0, 0, 0);
      c = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bl, c, 0, 0, 0);
      c = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bh, c, 0, 0, 0);
    } else if (mode == 1) {
      floatx4 t = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, bh, z, 0, 0, 0);
      t = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bl, t, 0, 0, 0);
      t = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bh, t, 0, 0, 0);
      c = c + t;
    } else {
      floatx4 t = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, bh, z, 0, 0, 0);
      t = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bl, t, 0, 0, 0);
      c = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bh, c, 0, 0, 0);
      c = c + t;
    }
  }
  for (int r = 0; r < 4; ++r) D[t * 256 + (4 * kg + r) * 16 + row] = c[r];
}

extern "C" int split_chain(const void* A, const void* B, float* D, int n_trial, int mode) {
  const size_t n = (size_t)n_trial * 2 * 16 * 512 * 2;
  void *dA, *dB;
  float* dD;
  if (hipMalloc(&dA, n) || hipMalloc(&dB, n) || hipMalloc((void**)&dD, (size_t)n_trial * 1024)) return 1;
  (void)hipMemcpy(dA, A, n, hipMemcpyHostToDevice);
  (void)hipMemcpy(dB, B, n, hipMemcpyHostToDevice);
  k_split_chain<<<n_trial, 64>>>((const _Float16*)dA, (const _Float16*)dB, dD, mode);
  const int err = hipDeviceSynchronize() != hipSuccess;
  (void)hipMemcpy(D, dD, (size_t)n_trial * 1024, hipMemcpyDeviceToHost);
  (void)hipFree(dA); (void)hipFree(dB); (void)hipFree(dD);
  return err;
}

typedef float float2v __attribute__((ext_vector_type(2)));
typedef _Float16 half2v __attribute__((ext_vector_type(2)));
// the split of dsr_mlp16.hpp: write_split's conversion (hi) and fma_mix remainder (lo)
__global__ void k_cvt(const float* x, _Float16* h, _Float16* l, int n) {
  const int i = 2 * (blockIdx.x * blockDim.x + threadIdx.x);
  if (i + 1 >= n) return;
  const float2v v = float2v{x[i], x[i + 1]};
  const half2v hv = __builtin_convertvector(v, half2v);
  const unsigned hb = __builtin_bit_cast(unsigned, hv);
  unsigned lb;
  asm("v_fma_mixlo_f16 %0, -%1, 1.0, %2 op_sel_hi:[1,0,0]" : "=v"(lb) : "v"(hb), "v"(v[0]));
  asm("v_fma_mixhi_f16 %0, -%1, 1.0, %2 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "+v"(lb) : "v"(hb), "v"(v[1]));
  const half2v lv = __builtin_bit_cast(half2v, lb);
  h[i] = hv[0]; h[i + 1] = hv[1];
  l[i] = lv[0]; l[i + 1] = lv[1];
}

extern "C" int cvt(const float* x, _Float16* h, _Float16* l, int n) {
  float* dx; _Float16 *dh, *dl;
  if (hipMalloc((void**)&dx, n * 4) || hipMalloc((void**)&dh, n * 2) || hipMalloc((void**)&dl, n * 2)) return 1;
  (void)hipMemcpy(dx, x, n * 4, hipMemcpyHostToDevice);
  k_cvt<<<(n / 2 + 255) / 256, 256>>>(dx, dh, dl, n);
  const int err = hipDeviceSynchronize() != hipSuccess;
  (void)hipMemcpy(h, dh, n * 2, hipMemcpyDeviceToHost);
  (void)hipMemcpy(l, dl, n * 2, hipMemcpyDeviceToHost);
  (void)hipFree(dx); (void)hipFree(dh); (void)hipFree(dl);
  return err;
}

extern "C" int probe(const void* A, const void* B, const float* C, float* D, int n_trial, int mode) {
  const size_t na = (size_t)n_trial * (mode == 2 ? 64 * 4 : 16 * 32 * (mode == 1 ? 2 : 1) * 2);
  void *dA, *dB;
  float *dC, *dD;
  if (hipMalloc(&dA, na) || hipMalloc(&dB, na) || hipMalloc((void**)&dC, n_trial * 1024) ||
      hipMalloc((void**)&dD, n_trial * 1024))
    return 1;
  hipMemcpy(dA, A, na, hipMemcpyHostToDevice);
  hipMemcpy(dB, B, na, hipMemcpyHostToDevice);
  hipMemcpy(dC, C, n_trial * 1024, hipMemcpyHostToDevice);
  k_probe<<<n_trial, 64>>>((const _Float16*)dA, (const _Float16*)dB, dC, dD, mode);
  const int err = hipDeviceSynchronize() != hipSuccess;
  hipMemcpy(D, dD, n_trial * 1024, hipMemcpyDeviceToHost);
  hipFree(dA); hipFree(dB); hipFree(dC); hipFree(dD);
  return err;
}

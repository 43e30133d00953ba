// dsr_mlp_lite.hpp — the one-product ("lite") decoder pass that classifies render samples.
//
// k_render only needs, for a ray sample, its occupancy 0.5 - clamp(sdf, +-th)/(2 th)
// (loss_utils.py:40-48) and whether |sdf| < th (loss.py:101): for sdf >= th the sample is
// exactly empty (o = 0), for sdf <= -th exactly full (o = 1), and only the samples in
// between need their SDF value.  The lite pass decodes every sample with one fp16 MFMA
// product (hi(W) . hi(H), fp32 accumulate: 1/3 of the split-fp16 MFMA work, half its
// weight bytes) on 128-point tiles (the hi image alone fits LDS twice as wide, halving
// the weight stream per point again), and
//   * writes its value to `dense` (a value outside the band has the class of the exact one),
//   * flags the ray dead when sdf <= -th - margin (certainly full: early termination),
//   * flags the sample for the exact split-fp16 pass when |sdf| < th + margin.
// The margin bounds the lite pass's error and calibrates itself per object: 0.02 in the
// first GN iteration, then max(0.005, 8 x the largest |lite - exact| the object's own
// re-decoded samples have shown so far) — the exact pass measures that error on every
// band sample it overwrites (max 8.5e-4 over 1.8M samples of 18 shapes offline,
// tools/cheap_error.py); a margin above 0.1 sends every sample to the exact pass.  The
// refined samples carry the exact values, so every occupancy, mask and de_do downstream
// is the split-fp16 one.
// Layout: tile = 128 points, 512 threads; wave w owns rows 64w..64w+63 as 4 x 8 blocks of
// 16x16 accumulators; LDS image H[128][528] fp16 (per-tile power-of-two scale as in
// dsr_mlp16.hpp); weights: the hi pieces of the split fragments (one 1 KiB wave-load per
// row block and k step).
#pragma once
#include "dsr_dev.hpp"
#include "dsr_mlp.hpp"
#include "dsr_mlp16.hpp"

namespace dsr {

constexpr int LTILE = 128;

struct LiteShared {
  _Float16 H[LTILE * PH];
  float xyz[LTILE * 4];
  float red[NWAVE * LTILE];
  float wmax[NWAVE];
};

// acc[4][8] = hi(A rows of this wave) . hi(H) over K = 32*T
template <bool PRIO>
__device__ __forceinline__ void gemm_lite(const half8* __restrict__ A, int T, const _Float16* H,
                                          floatx4 (&acc)[4][8], int lane) {
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int cb = 0; cb < 8; ++cb) acc[q][cb] = floatx4{0.f, 0.f, 0.f, 0.f};
  const _Float16* B = H + (lane & 15) * PH + 8 * (lane >> 4);
  half8 a0[4], a1[4], b0[8], b1[8];
#pragma unroll
  for (int q = 0; q < 4; ++q) a0[q] = A[((q * T) * 2) * 64 + lane];
#pragma unroll
  for (int cb = 0; cb < 8; ++cb) b0[cb] = *reinterpret_cast<const half8*>(B + cb * 16 * PH);
  for (int t = 0; t < T; t += 2) {
#pragma unroll
    for (int q = 0; q < 4; ++q) a1[q] = A[((q * T + t + 1) * 2) * 64 + lane];
#pragma unroll
    for (int cb = 0; cb < 8; ++cb) b1[cb] = *reinterpret_cast<const half8*>(B + cb * 16 * PH + 32 * (t + 1));
    if (PRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int cb = 0; cb < 8; ++cb)
        acc[q][cb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a0[q], b0[cb], acc[q][cb], 0, 0, 0);
    if (PRIO) __builtin_amdgcn_s_setprio(0);
    if (t + 2 < T) {
#pragma unroll
      for (int q = 0; q < 4; ++q) a0[q] = A[((q * T + t + 2) * 2) * 64 + lane];
#pragma unroll
      for (int cb = 0; cb < 8; ++cb) b0[cb] = *reinterpret_cast<const half8*>(B + cb * 16 * PH + 32 * (t + 2));
    }
    if (PRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int cb = 0; cb < 8; ++cb)
        acc[q][cb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a1[q], b1[cb], acc[q][cb], 0, 0, 0);
    if (PRIO) __builtin_amdgcn_s_setprio(0);
  }
}

// block max of m (>= 0) -> power-of-two scale exponent; contains the barrier that ends
// every wave's reads of H for the GEMM just finished
__device__ __forceinline__ int lite_block_scale(float m, float* wmax, int w, int lane) {
  m = wave_max(m);
  if (lane == 0) wmax[w] = m;
  __syncthreads();
  float mm = wmax[0];
#pragma unroll
  for (int k = 1; k < NWAVE; ++k) mm = fmaxf(mm, wmax[k]);
  return act_scale_exp(mm);
}

__device__ __forceinline__ void lite_write(floatx4 (&acc)[4][8], int s, _Float16* H, int w, int lane) {
  const int g = lane >> 4, c = lane & 15;
  const float sc = ldexpf(1.f, s);
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int n0 = 64 * w + 16 * q + 4 * g;
#pragma unroll
    for (int cb = 0; cb < 8; ++cb) {
      half4 h;
#pragma unroll
      for (int r = 0; r < 4; ++r) h[r] = (_Float16)(accr(acc[q][cb], r) * sc);
      *reinterpret_cast<half4*>(H + (16 * cb + c) * PH + n0) = h;
    }
  }
}

template <bool PRIO>
__global__ __launch_bounds__(512) void k_mlp_fwd_lite(DevDecoder D, const Tile* __restrict__ tiles,
                                                      const int* __restrict__ n_tiles,
                                                      const ObjDesc* __restrict__ desc,
                                                      const float4* __restrict__ cand,
                                                      const float* __restrict__ bias0f,
                                                      const float* __restrict__ bias4f,
                                                      float* __restrict__ dense, ErtArgs E) {
  __shared__ LiteShared sm;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, c = lane & 15;
  const int nt = *n_tiles;
  for (int ti = blockIdx.x; ti < nt; ti += gridDim.x) {
    const Tile tl = tiles[ti];
    const ObjDesc d = desc[tl.obj];
    if (tid < LTILE) {
      const float4 v = (tid < tl.count) ? cand[d.cand_off + tl.start + tid] : make_float4(0.f, 0.f, 0.f, 0.f);
      sm.xyz[tid * 4 + 0] = v.x; sm.xyz[tid * 4 + 1] = v.y;
      sm.xyz[tid * 4 + 2] = v.z; sm.xyz[tid * 4 + 3] = v.w;
    }
    __syncthreads();
    floatx4 acc[4][8];
    int sa;
    // ---- lin0 (3 inputs, fp32 VALU) into the accumulator layout
    {
      const float* bias0 = bias0f + tl.obj * HID;
      float m = 0.f;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int n0 = 64 * w + 16 * q + 4 * g;
        const float4 bb = *reinterpret_cast<const float4*>(bias0 + n0);
        float wx[12];
#pragma unroll
        for (int i = 0; i < 12; ++i) wx[i] = D.W0x[n0 * 3 + i];
#pragma unroll
        for (int cb = 0; cb < 8; ++cb) {
          const int p = 16 * cb + c;
          const float x = sm.xyz[p * 4 + 0], y = sm.xyz[p * 4 + 1], z = sm.xyz[p * 4 + 2];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float a = fetch4(bb, r) + ((wx[3 * r] * x + wx[3 * r + 1] * y) + wx[3 * r + 2] * z);
            const float h = fmaxf(a, 0.f);
            acc[q][cb][r] = h;
            m = fmaxf(m, h);
          }
        }
      }
      sa = lite_block_scale(m, sm.wmax, w, lane);
      lite_write(acc, sa, sm.H, w, lane);
    }
    __syncthreads();
    // ---- lin1..lin6
    for (int l = 1; l <= 6; ++l) {
      const int T = D.Kf[l] / 32;
      gemm_lite<PRIO>(wfrag(D.Wh_raw[l], w, T), T, sm.H, acc, lane);
      const float usc = ldexpf(1.f, -(D.sw[l] + sa));
      const float* bias = (l == 4) ? bias4f + tl.obj * HID : D.bias[l];
      float m = 0.f;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int n0 = 64 * w + 16 * q + 4 * g;
        const float4 bb = *reinterpret_cast<const float4*>(bias + n0);
#pragma unroll
        for (int cb = 0; cb < 8; ++cb) {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            float x = fmaxf(__builtin_fmaf(accr(acc[q][cb], r), usc, fetch4(bb, r)), 0.f);
            if (l == 3 && n0 == 444 && r > 0) x = sm.xyz[(16 * cb + c) * 4 + (r - 1)];   // lin4 input: h3 | xyz
            acc[q][cb][r] = x;
            m = fmaxf(m, fabsf(x));           // (xyz rows of lin3 may be negative)
          }
        }
      }
      sa = lite_block_scale(m, sm.wmax, w, lane);
      lite_write(acc, sa, sm.H, w, lane);
      __syncthreads();
    }
    // ---- lin7 + relu, lin8 dot product, tanh
    {
      const int T = D.Kf[7] / 32;
      gemm_lite<PRIO>(wfrag(D.Wh_raw[7], w, T), T, sm.H, acc, lane);
      const float usc = ldexpf(1.f, -(D.sw[7] + sa));
      float part[8];
#pragma unroll
      for (int cb = 0; cb < 8; ++cb) part[cb] = 0.f;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int n0 = 64 * w + 16 * q + 4 * g;
        const float4 bb = *reinterpret_cast<const float4*>(D.bias[7] + n0);
        const float4 w8 = *reinterpret_cast<const float4*>(D.W8 + n0);
#pragma unroll
        for (int cb = 0; cb < 8; ++cb)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float v = fmaxf(__builtin_fmaf(accr(acc[q][cb], r), usc, fetch4(bb, r)), 0.f);
            part[cb] = __builtin_fmaf(fetch4(w8, r), v, part[cb]);
          }
      }
#pragma unroll
      for (int cb = 0; cb < 8; ++cb) {
        float s = part[cb];
        s += __shfl_xor(s, 16);
        s += __shfl_xor(s, 32);
        if (g == 0) sm.red[w * LTILE + 16 * cb + c] = s;
      }
    }
    __syncthreads();
    if (tid < tl.count) {
      float s = sm.red[tid];
      for (int k = 1; k < NWAVE; ++k) s += sm.red[k * LTILE + tid];
      float y = tanhf(s + D.b8);
      const float px = sm.xyz[tid * 4 + 0], py = sm.xyz[tid * 4 + 1], pz = sm.xyz[tid * 4 + 2];
      if (px != px || py != py || pz != pz || bias0f[tl.obj * HID] != bias0f[tl.obj * HID])
        y = __builtin_nanf("");
      const int idx = __float_as_int(sm.xyz[tid * 4 + 3]);
      const float margin = E.st[tl.obj].lite_margin;
      dense[d.cand_off + idx] = y;
      if (y <= E.nth - margin) E.dead[d.ray_off + idx / E.M] = 1;            // certainly full
      else if (!(y >= -E.nth + margin)) E.refine[d.cand_off + idx] = 1;      // band (or NaN)
    }
    __syncthreads();
  }
}

}  // namespace dsr

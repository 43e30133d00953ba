// dsr_mlp.hpp — DeepSDF decoder on CDNA4 fp32 MFMA (v_mfma_f32_16x16x4_f32).
//
// Restates deep_sdf/deep_sdf_decoder.py:75-110 (forward) and the autograd input
// Jacobian taken by reconstruct/loss_utils.py:82-113 (get_batch_sdf_jacobian) as
// fused, persistent, tile-per-workgroup kernels:
//
//   * a workgroup = 8 waves = 512 threads owns a tile of 64 points;
//   * the activation image H[point][neuron] (64 x 512 fp32, pitch 520) lives in LDS;
//   * every layer is Out[512 x 64] = W[512 x K] . H[K x 64]: wave w computes rows
//     64w..64w+63 for all 64 points = 4 x 4 blocks of 16x16 accumulators (64 VGPRs);
//   * the A operand (weights) streams from L2 in a pre-packed fragment layout (one
//     1 KiB coalesced dwordx4 wave-load per 16x16 block per 16 k), double-buffered in
//     registers; the B operand (activations) is read from LDS with ds_read_b128;
//   * the k order inside a 16-wide step is permuted (lane group g, MFMA sub-step j
//     -> neuron 16t+4g+j) identically for A and B, so each lane's A and B are a
//     single float4 each;
//   * the latent code is constant per object: its lin0/lin4 columns are folded
//     into a per-object bias (k_fold_bias), so lin0 is a 3-input VALU layer and
//     lin4 a 448-deep GEMM (445 h3 + 3 xyz);
//   * lin8 (512 -> 1) + tanh is a dot product fused into lin7's epilogue;
//   * the Jacobian kernel keeps the ReLU masks as bits in registers (the backward
//     GEMM W_l^T g_l produces rows in exactly the forward layout of layer l-1) and
//     streams pre-packed W_l^T fragments.
#pragma once
#include "dsr_dev.hpp"

namespace dsr {

constexpr int H_FLOATS = TILE * PITCH;          // 33280 floats = 133,120 B

template <int NQ>
__device__ __forceinline__ void mfma_step(const float4 (&a)[NQ], const float4 (&b)[4],
                                          floatx4 (&acc)[NQ][4]) {
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int q = 0; q < NQ; ++q)
#pragma unroll
      for (int cb = 0; cb < 4; ++cb)
        acc[q][cb] = __builtin_amdgcn_mfma_f32_16x16x4f32(fetch4(a[q], j), fetch4(b[cb], j),
                                                          acc[q][cb], 0, 0, 0);
}

// acc[q][cb] (16x16 block: rows 16(rb0+q).., points 16cb..) = A(rows) . H(points)
// A: packed fragments of this wave's first row block: element (q, t) at A[(q*T+t)*64+lane].
template <int NQ>
__device__ __forceinline__ void gemm_tile(const float4* __restrict__ A, int T,
                                          const float* __restrict__ Hs,
                                          floatx4 (&acc)[NQ][4], int lane) {
#pragma unroll
  for (int q = 0; q < NQ; ++q)
#pragma unroll
    for (int cb = 0; cb < 4; ++cb) acc[q][cb] = floatx4{0.f, 0.f, 0.f, 0.f};
  const float* Bp = Hs + (lane & 15) * PITCH + 4 * (lane >> 4);
  float4 a0[NQ], a1[NQ];
#pragma unroll
  for (int q = 0; q < NQ; ++q) a0[q] = A[(q * T) * 64 + lane];
  for (int t = 0; t < T; t += 2) {
#pragma unroll
    for (int q = 0; q < NQ; ++q) a1[q] = A[(q * T + t + 1) * 64 + lane];
    float4 b[4];
#pragma unroll
    for (int cb = 0; cb < 4; ++cb)
      b[cb] = *reinterpret_cast<const float4*>(Bp + cb * 16 * PITCH + 16 * t);
    mfma_step<NQ>(a0, b, acc);
    const int tn = (t + 2 < T) ? t + 2 : T - 1;      // clamped prefetch (no branch)
#pragma unroll
    for (int q = 0; q < NQ; ++q) a0[q] = A[(q * T + tn) * 64 + lane];
#pragma unroll
    for (int cb = 0; cb < 4; ++cb)
      b[cb] = *reinterpret_cast<const float4*>(Bp + cb * 16 * PITCH + 16 * (t + 1));
    mfma_step<NQ>(a1, b, acc);
  }
}

// Same GEMM with the B fragments (LDS) of the next 16-k step loaded before the MFMAs of
// the current one (+16 VGPRs), so ds_read latency never sits in front of an MFMA.
template <int NQ, bool PRIO>
__device__ __forceinline__ void gemm_tile_pf(const float4* __restrict__ A, int T,
                                             const float* __restrict__ Hs,
                                             floatx4 (&acc)[NQ][4], int lane) {
#pragma unroll
  for (int q = 0; q < NQ; ++q)
#pragma unroll
    for (int cb = 0; cb < 4; ++cb) acc[q][cb] = floatx4{0.f, 0.f, 0.f, 0.f};
  const float* Bp = Hs + (lane & 15) * PITCH + 4 * (lane >> 4);
  float4 a0[NQ], a1[NQ], b0[4], b1[4];
#pragma unroll
  for (int q = 0; q < NQ; ++q) a0[q] = A[(q * T) * 64 + lane];
#pragma unroll
  for (int cb = 0; cb < 4; ++cb) b0[cb] = *reinterpret_cast<const float4*>(Bp + cb * 16 * PITCH);
  for (int t = 0; t < T; t += 2) {
#pragma unroll
    for (int q = 0; q < NQ; ++q) a1[q] = A[(q * T + t + 1) * 64 + lane];
#pragma unroll
    for (int cb = 0; cb < 4; ++cb)
      b1[cb] = *reinterpret_cast<const float4*>(Bp + cb * 16 * PITCH + 16 * (t + 1));
    if (PRIO) __builtin_amdgcn_s_setprio(1);
    mfma_step<NQ>(a0, b0, acc);
    if (PRIO) __builtin_amdgcn_s_setprio(0);
    const int tn = (t + 2 < T) ? t + 2 : T - 1;
#pragma unroll
    for (int q = 0; q < NQ; ++q) a0[q] = A[(q * T + tn) * 64 + lane];
#pragma unroll
    for (int cb = 0; cb < 4; ++cb)
      b0[cb] = *reinterpret_cast<const float4*>(Bp + cb * 16 * PITCH + 16 * tn);
    if (PRIO) __builtin_amdgcn_s_setprio(1);
    mfma_step<NQ>(a1, b1, acc);
    if (PRIO) __builtin_amdgcn_s_setprio(0);
  }
}

// Soft barrier among the workgroups that share the label blockIdx % 8 (the dispatcher's
// XCD round robin, MI355X_MICROARCH.md §Workgroup dispatch): keeps each XCD's workgroups
// on the same layer so the layer's 1 MB of weights is an L2 hit for all but the first.
// Purely a speed device: no data is handed over, the spin is bounded, and a wrong
// placement guess only costs time.
__device__ __forceinline__ void group_soft_sync(unsigned* ctr, int round) {
  __syncthreads();
  if (threadIdx.x == 0) {
    const int g = blockIdx.x & 7;
    const unsigned gs = (gridDim.x - g + 7) / 8;
    unsigned* c = ctr + g * 32;
    const unsigned target = (unsigned)(round + 1) * gs;
    atomicAdd(c, 1u);
    for (int spin = 0; spin < (1 << 16); ++spin) {
      if (atomicAdd(c, 0u) >= target) break;
      __builtin_amdgcn_s_sleep(4);
    }
  }
  __syncthreads();
}

// ReLU that keeps torch's NaN propagation (torch.relu(nan) == nan).
__device__ __forceinline__ float relu_t(float a) { return a > 0.f ? a : (a == a ? 0.f : a); }
// threshold_backward keeps the gradient where NOT (out <= 0)
__device__ __forceinline__ bool relu_pass(float out) { return !(out <= 0.f); }

__device__ __forceinline__ float accr(const floatx4& v, int r) {
  return r == 0 ? v[0] : (r == 1 ? v[1] : (r == 2 ? v[2] : v[3]));
}

// lin0 on VALU in the accumulator layout: h0[n][p] = relu(b0'[n] + W0x[n] . xyz_p).
__device__ __forceinline__ void layer0_fwd(const DevDecoder& D, const float* __restrict__ bias0,
                                           const float* __restrict__ xyz, float* Hs, int w,
                                           int lane, uint64_t& mask) {
  const int g = lane >> 4, c = lane & 15;
  mask = 0;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int n0 = 64 * w + 16 * q + 4 * g;
    const float4 bb = *reinterpret_cast<const float4*>(bias0 + n0);
    float wx[12];
#pragma unroll
    for (int i = 0; i < 12; ++i) wx[i] = D.W0x[n0 * 3 + i];
#pragma unroll
    for (int cb = 0; cb < 4; ++cb) {
      const int p = 16 * cb + c;
      const float x = xyz[p * 4 + 0], y = xyz[p * 4 + 1], z = xyz[p * 4 + 2];
      float v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float a = fetch4(bb, r) + ((wx[3 * r] * x + wx[3 * r + 1] * y) + wx[3 * r + 2] * z);
        v[r] = relu_t(a);
        if (relu_pass(v[r])) mask |= 1ull << ((q * 4 + cb) * 4 + r);
      }
      *reinterpret_cast<float4*>(Hs + p * PITCH + n0) = make_float4(v[0], v[1], v[2], v[3]);
    }
  }
}

// Epilogue of a forward hidden layer: relu(acc + b) -> Hs (+ mask bits).  For lin3 the
// padded rows 445..447 are overwritten with the point's xyz: they become the 3 xyz
// columns of lin4's 448-deep input (the 64 code columns are folded into bias4).
__device__ __forceinline__ void epi_fwd(floatx4 (&acc)[4][4], const float* __restrict__ bias,
                                        float* Hs, const float* __restrict__ xyz, int w,
                                        int lane, uint64_t& mask, bool is_l3, int l3) {
  const int g = lane >> 4, c = lane & 15;
  mask = 0;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int n0 = 64 * w + 16 * q + 4 * g;
    const float4 bb = *reinterpret_cast<const float4*>(bias + n0);
#pragma unroll
    for (int cb = 0; cb < 4; ++cb) {
      const int p = 16 * cb + c;
      float v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        v[r] = relu_t(accr(acc[q][cb], r) + fetch4(bb, r));
        if (relu_pass(v[r])) mask |= 1ull << ((q * 4 + cb) * 4 + r);
      }
      if (is_l3 && n0 == l3 - 1) {       // rows l3..l3+2 (445..447 at code_len 64) <- x,y,z
        v[1] = xyz[p * 4 + 0];
        v[2] = xyz[p * 4 + 1];
        v[3] = xyz[p * 4 + 2];
      }
      *reinterpret_cast<float4*>(Hs + p * PITCH + n0) = make_float4(v[0], v[1], v[2], v[3]);
    }
  }
}

// lin7 epilogue fused with lin8 (512 -> 1): per-wave partial dot products -> red[w][p].
// xyz_in_all: lin8's input rows 509..511 (wave 7, block 3, quad 3, r 1..3) are the point's
// x, y, z (xyz: the tile's float4 points), not lin7 outputs — their mask bits stay the ReLU's (0)
__device__ __forceinline__ void epi_l7(floatx4 (&acc)[4][4], const DevDecoder& D, float* red,
                                       int w, int lane, uint64_t& mask, const float* xyz = nullptr,
                                       bool with_bias = true) {   // false: acc holds LN(lin7) (ln_l7)
  const int g = lane >> 4, c = lane & 15;
  mask = 0;
  float part[4] = {0.f, 0.f, 0.f, 0.f};
  const bool xr = D.xyz_all && xyz != nullptr && w == 7;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int n0 = 64 * w + 16 * q + 4 * g;
    const float4 bb = with_bias ? *reinterpret_cast<const float4*>(D.bias[7] + n0) : make_float4(0.f, 0.f, 0.f, 0.f);
    const float4 w8 = *reinterpret_cast<const float4*>(D.W8 + n0);
#pragma unroll
    for (int cb = 0; cb < 4; ++cb) {
      float4 p = make_float4(0.f, 0.f, 0.f, 0.f);
      const bool on = xr && q == 3 && g == 3;
      if (q == 3 && xr) p = *reinterpret_cast<const float4*>(xyz + (16 * cb + c) * 4);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float v = relu_t(accr(acc[q][cb], r) + fetch4(bb, r));
        if (relu_pass(v)) mask |= 1ull << ((q * 4 + cb) * 4 + r);
        if (r >= 1) v = on ? (r == 1 ? p.x : (r == 2 ? p.y : p.z)) : v;
        part[cb] = __builtin_fmaf(fetch4(w8, r), v, part[cb]);
      }
    }
  }
#pragma unroll
  for (int cb = 0; cb < 4; ++cb) {
    float s = part[cb];
    s += xor_lane(s, lane, 16);
    s += xor_lane(s, lane, 32);
    if (g == 0) red[w * 64 + 16 * cb + c] = s;
  }
}

// Backward epilogue: g_{l-1} = acc (.) relu'(layer l-1) -> Hs.
__device__ __forceinline__ void epi_bwd(floatx4 (&acc)[4][4], float* Hs, int w, int lane,
                                        uint64_t mask) {
  const int g = lane >> 4, c = lane & 15;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int n0 = 64 * w + 16 * q + 4 * g;
#pragma unroll
    for (int cb = 0; cb < 4; ++cb) {
      const int p = 16 * cb + c;
      float v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r)
        v[r] = ((mask >> ((q * 4 + cb) * 4 + r)) & 1ull) ? accr(acc[q][cb], r) : 0.f;
      *reinterpret_cast<float4*>(Hs + p * PITCH + n0) = make_float4(v[0], v[1], v[2], v[3]);
    }
  }
}

// lin4^T epilogue: rows 0..444 -> g3 (masked) into Hs, rows 445..511 (= d/d[code, xyz]
// through the latent skip, deep_sdf_decoder.py:87-88) -> gin[p][n-445]; Hs rows
// 445..447 are zeroed (they are K padding of the lin3^T GEMM).
constexpr int GIN_PITCH = 68;
__device__ __forceinline__ void epi_bwd_l4(floatx4 (&acc)[4][4], float* Hs, float* gin, int w,
                                           int lane, uint64_t mask3, int l3, int kb3) {
  const int g = lane >> 4, c = lane & 15;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int n0 = 64 * w + 16 * q + 4 * g;
#pragma unroll
    for (int cb = 0; cb < 4; ++cb) {
      const int p = 16 * cb + c;
      float v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = n0 + r;
        const float a = accr(acc[q][cb], r);
        if (n < l3) {
          v[r] = ((mask3 >> ((q * 4 + cb) * 4 + r)) & 1ull) ? a : 0.f;
        } else {
          v[r] = 0.f;
          gin[p * GIN_PITCH + gin_slot(n, l3)] = a;
        }
      }
      if (n0 < kb3)
        *reinterpret_cast<float4*>(Hs + p * PITCH + n0) = make_float4(v[0], v[1], v[2], v[3]);
    }
  }
}

}  // namespace dsr

// dsr_kernels.hpp — the device-resident Gauss-Newton iteration of
// Optimizer.reconstruct_object (reconstruct/optimizer.py:90-205) for a batch of
// independent objects.  One iteration = 9 + 3 x (render passes) launches per object group on
// the chunked path (one group), 12 + 3 x (render passes) otherwise, none of which needs the host:
//
//   k_iter_begin   optimizer.py:122-128  t_cam_obj, scale, linspace depths, bg depth,
//                                        + code folded into lin0 / lin4 biases
//   per render pass (early ray termination, exact — see k_sample_pass):
//   k_sample_scan / k_sample_count + k_sample_emit
//                  loss.py:71-88         ray samples -> object frame -> |x|<1 ->
//                                        (ray, depth)-ordered compaction of live rays
//   k_tiles_fwd    —                     tiles over the pass's samples (chunked path: built
//                                        by an extra workgroup of k_sample_emit / k_refine_emit)
//   k_mlp_fwd      loss.py:91-92         decode_sdf (MFMA), flags terminated rays
//   k_render       loss.py:97-150        occupancy, transmittance cumprod, rendered
//                                        depth, de_do, K-compaction, residual clamp
//   k_tiles_jac    —                     tiles over N surface pts + K render pts
//   k_mlp_jac      loss.py:22-43,157-164 fwd + analytic input Jacobian (MFMA), Sim(3)
//                  loss_utils.py:176-195 point Jacobian, Huber (loss_utils.py:246-275),
//                  optimizer.py:163-169  per-tile J^T J, J^T r~, sum r~^2
//   k_solve        optimizer.py:131-194  reduce, damp, rotation prior, fp64 Cholesky solve,
//                                        exp_sim3, pose/code update, failure exits
#pragma once
#include "dsr_dev.hpp"
#include "dsr_mlp.hpp"
#include "dsr_mlp16.hpp"
#include "dsr_mlp_lite.hpp"
#include "../../include/dsr.h"

// wave-wide 64-bit max (ockl DPP reduction; declared by HIP only under
// HIP_ENABLE_EXTRA_WARP_SYNC_TYPES)
extern "C" __device__ __attribute__((const)) unsigned long long __ockl_wfred_max_u64(unsigned long long);

namespace dsr {

// ------------------------------------------------------------------------------------
// small fp32 linear algebra (single thread), mirroring torch CPU fp32 semantics
// ------------------------------------------------------------------------------------
// LU with partial pivoting (first max, LAPACK getrf), multipliers by reciprocal (sgetf2).
// Fully unrolled with the row swap as selects, so every index is static and the matrix stays
// in registers (a swap through a run-time pivot index would put it in scratch memory).
template <int N>
__device__ __forceinline__ void lu_small(float (&a)[N][N], int (&piv)[N]) {
#pragma unroll
  for (int k = 0; k < N; ++k) {
    int p = k;
    float best = fabsf(a[k][k]);
#pragma unroll
    for (int r = k + 1; r < N; ++r)
      if (fabsf(a[r][k]) > best) { best = fabsf(a[r][k]); p = r; }
    piv[k] = p;
#pragma unroll
    for (int r = k + 1; r < N; ++r) {
      const bool sw = (p == r);
#pragma unroll
      for (int c = 0; c < N; ++c) {
        const float t = a[k][c];
        a[k][c] = sw ? a[r][c] : t;
        a[r][c] = sw ? t : a[r][c];
      }
    }
    const float rc = 1.0f / a[k][k];
#pragma unroll
    for (int r = k + 1; r < N; ++r) a[r][k] = a[r][k] * rc;
#pragma unroll
    for (int r = k + 1; r < N; ++r)
#pragma unroll
      for (int c = k + 1; c < N; ++c) a[r][c] = __builtin_fmaf(-a[r][k], a[k][c], a[r][c]);
  }
}

template <int N>
__device__ __forceinline__ void inv_small(const float* m, float* out) {   // torch.inverse (getrf + getrs(I))
  float a[N][N];
  int piv[N];
#pragma unroll
  for (int i = 0; i < N; ++i)
#pragma unroll
    for (int j = 0; j < N; ++j) a[i][j] = m[i * N + j];
  lu_small<N>(a, piv);
#pragma unroll
  for (int col = 0; col < N; ++col) {
    float x[N];
#pragma unroll
    for (int i = 0; i < N; ++i) x[i] = (i == col) ? 1.f : 0.f;
#pragma unroll
    for (int k = 0; k < N; ++k)       // row interchanges, as selects (static indices)
#pragma unroll
      for (int r = k + 1; r < N; ++r) {
        const bool sw = (piv[k] == r);
        const float t = x[k];
        x[k] = sw ? x[r] : t;
        x[r] = sw ? t : x[r];
      }
#pragma unroll
    for (int i = 0; i < N; ++i)
#pragma unroll
      for (int l = 0; l < i; ++l) x[i] = __builtin_fmaf(-a[i][l], x[l], x[i]);
#pragma unroll
    for (int i = N - 1; i >= 0; --i) {
#pragma unroll
      for (int l = i + 1; l < N; ++l) x[i] = __builtin_fmaf(-a[i][l], x[l], x[i]);
      x[i] = x[i] / a[i][i];
    }
#pragma unroll
    for (int i = 0; i < N; ++i) out[i * N + col] = x[i];
  }
}

__device__ __forceinline__ float det3(const float* m4 /*4x4, uses [:3,:3]*/) {   // torch.det via LU
  float a[3][3];
  int piv[3];
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) a[i][j] = m4[i * 4 + j];
  lu_small<3>(a, piv);
  float d = (a[0][0] * a[1][1]) * a[2][2];
  int sw = (piv[0] != 0) + (piv[1] != 1);
  return (sw & 1) ? -d : d;
}

__device__ void mm4(const float* A, const float* B, float* C) {
  float t[16];
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 4; ++j) {
      float s = 0.f;
      for (int k = 0; k < 4; ++k) s = s + A[i * 4 + k] * B[k * 4 + j];
      t[i * 4 + j] = s;
    }
  for (int i = 0; i < 16; ++i) C[i] = t[i];
}

// exp_sim3 (loss_utils.py:198-243) in fp32, branch structure included
// (theta<=1e-8 & s==0 / s!=0; c = 0 when s <= eps, also for negative s).
__device__ void exp_sim3_dev(const float* x, float* out) {
  const float v0 = x[0], v1 = x[1], v2 = x[2], w0 = x[3], w1 = x[4], w2 = x[5], s = x[6];
  const float W[9] = {0.f, -w2, w1, w2, 0.f, -w0, -w1, w0, 0.f};
  float W2[9];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j)
      W2[i * 3 + j] = (W[i * 3 + 0] * W[0 * 3 + j] + W[i * 3 + 1] * W[1 * 3 + j]) + W[i * 3 + 2] * W[2 * 3 + j];
  const float theta = sqrtf((w0 * w0 + w1 * w1) + w2 * w2);
  const float t2 = theta * theta;
  const float st = sinf(theta), ct = cosf(theta);
  const float es = expf(s);
  const float s2 = s * s;
  float ew[9], J[9];
  const float I3[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
  if (theta <= 1e-8f) {
    if (s == 0.f) {
      for (int i = 0; i < 9; ++i) { ew[i] = I3[i]; J[i] = I3[i]; }
    } else {
      const float c = (es - 1.f) / s;
      for (int i = 0; i < 9; ++i) { ew[i] = I3[i]; J[i] = c * I3[i]; }
    }
  } else {
    for (int i = 0; i < 9; ++i) ew[i] = (I3[i] + W[i] * st / theta) + W2[i] * (1.f - ct) / t2;
    const float a = es * st, b = es * ct;
    const float c = (s <= 1e-8f) ? 0.f : (es - 1.f) / s;
    const float k1 = (a * s + (1.f - b) * theta) / (s2 + t2);
    const float k2 = c - ((b - 1.f) * s + a * theta) / (s2 + t2);
    for (int i = 0; i < 9; ++i) J[i] = (c * I3[i] + k1 * W[i] / theta) + k2 * W2[i] / t2;
  }
  for (int i = 0; i < 16; ++i) out[i] = (i % 5 == 0) ? 1.f : 0.f;
  for (int i = 0; i < 3; ++i) {
    for (int j = 0; j < 3; ++j) out[i * 4 + j] = es * ew[i * 3 + j];
    out[i * 4 + 3] = (J[i * 3 + 0] * v0 + J[i * 3 + 1] * v1) + J[i * 3 + 2] * v2;
  }
}

// exp_se3 (loss_utils.py:139-173) in fp32: x = (v, w), theta <= 1e-8 -> identity rotation.
__device__ void exp_se3_dev(const float* x, float* out) {
  const float v0 = x[0], v1 = x[1], v2 = x[2], w0 = x[3], w1 = x[4], w2 = x[5];
  const float W[9] = {0.f, -w2, w1, w2, 0.f, -w0, -w1, w0, 0.f};
  float W2[9];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j)
      W2[i * 3 + j] = (W[i * 3 + 0] * W[0 * 3 + j] + W[i * 3 + 1] * W[1 * 3 + j]) + W[i * 3 + 2] * W[2 * 3 + j];
  const float theta = sqrtf((w0 * w0 + w1 * w1) + w2 * w2);
  const float t2 = theta * theta, t3 = t2 * theta;
  const float st = sinf(theta), ct = cosf(theta);
  const float I3[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
  float ew[9], J[9];
  if (theta <= 1e-8f) {
    for (int i = 0; i < 9; ++i) { ew[i] = I3[i]; J[i] = I3[i]; }
  } else {
    for (int i = 0; i < 9; ++i) ew[i] = (I3[i] + W[i] * st / theta) + W2[i] * (1.f - ct) / t2;
    const float k1 = (1.f - ct) / t2, k2 = (theta - st) / t3;
    for (int i = 0; i < 9; ++i) J[i] = (I3[i] + k1 * W[i]) + k2 * W2[i];
  }
  for (int i = 0; i < 16; ++i) out[i] = (i % 5 == 0) ? 1.f : 0.f;
  for (int i = 0; i < 3; ++i) {
    for (int j = 0; j < 3; ++j) out[i * 4 + j] = ew[i * 3 + j];
    out[i * 4 + 3] = (J[i * 3 + 0] * v0 + J[i * 3 + 1] * v1) + J[i * 3 + 2] * v2;
  }
}


// ------------------------------------------------------------------------------------
// state init / per-iteration prologue
// ------------------------------------------------------------------------------------
__global__ void k_init_state(int n_obj, const float* __restrict__ t_in, const int* __restrict__ is_oc,
                             const float* __restrict__ z_in, ObjState* st, float* zbuf, int iters) {
  const int o = blockIdx.x;
  if (o >= n_obj) return;
  if (threadIdx.x < CODE) zbuf[o * CODE + threadIdx.x] = z_in[o * CODE + threadIdx.x];
  if (threadIdx.x == 0) {
    ObjState& S = st[o];
    if (is_oc[o]) {
      for (int i = 0; i < 16; ++i) S.T[i] = t_in[o * 16 + i];
    } else {
      inv_small<4>(t_in + o * 16, S.T);      // optimizer.py:105-106
    }
    S.loss = 0.f;                              // optimizer.py:119
    // zero iterations: the loop body never runs and the reference returns the input pose
    // and code with is_good=True, loss 0. (optimizer.py:120, 201-205)
    S.status = iters > 0 ? ST_RUNNING : ST_DONE;
    S.fail_reason = 0;
    S.iters_done = 0;
    S.n_valid = S.k = 0;
    S.sdf_loss = S.render_loss = 0.f;
    S.lite_margin = S.lite_err = 0.f;
    S.n_audit = S.lite_viol = S.lite_viol_total = S.lite_redo = 0;
  }
}

// optimizer.py:122-128 and the code fold of lin0 / lin4.
__global__ __launch_bounds__(512) void k_iter_begin(int n_obj, const ObjDesc* __restrict__ desc, ObjState* st,
                             const float* __restrict__ zbuf, DevDecoder D, GNParams P,
                             float* __restrict__ bias0f, float* __restrict__ bias4f,
                             float* __restrict__ dobs) {
  const int o = blockIdx.x;
  ObjState& S = st[o];
  if (S.status != ST_RUNNING) return;
  const int tid = threadIdx.x;
  __shared__ float z[CODE];
  if (tid < CODE) z[tid] = zbuf[o * CODE + tid];
  __syncthreads();
  for (int n = tid; n < HID; n += blockDim.x) {
    float s0 = 0.f, s4 = 0.f;
    for (int k = 0; k < CODE; ++k) {
      s0 = __builtin_fmaf(D.W0z[k * HID + n], z[k], s0);
      s4 = __builtin_fmaf(D.W4z[k * HID + n], z[k], s4);
    }
    bias0f[o * HID + n] = D.bias[0][n] + s0;
    bias4f[o * HID + n] = D.bias[4][n] + s4;
  }
  if (tid == 0) {
    float tco[16];                                             // (registers; S.Tco written once)
    inv_small<4>(S.T, tco);                                    // :122
#pragma unroll
    for (int i = 0; i < 16; ++i) S.Tco[i] = tco[i];
    const float scale = powf(det3(tco), 0.33333334f);          // :123 det ** (1/3)
    const float dmin = tco[11] - 1.0f * scale;                 // :124
    const float dmax = tco[11] + 1.0f * scale;
    const int M = P.M;
    const float step = (dmax - dmin) / (float)(M - 1);         // torch.linspace (CPU, fp32)
    const int half = M / 2;
    for (int i = 0; i < M; ++i)
      S.depths[i] = (i < half) ? __builtin_fmaf(step, (float)i, dmin)
                               : __builtin_fmaf(-step, (float)(M - 1 - i), dmax);
    S.dmin = S.depths[0];
    S.dmax = S.depths[M - 1];
    S.delta_d = (S.depths[M - 1] - S.depths[0]) / (float)(M - 1);   // loss.py:140
    S.bg_depth = 1.1f * dmax;                                  // :128
    S.n_valid = 0;
    S.k = 0;
    S.n_emit = S.n_eval = S.n_refine = 0;
    S.n_audit = S.lite_viol = 0;
    if (desc[o].n_rays == 0) {                          // no in-ball samples: loss.py:86-88 (the
      S.status = ST_FAIL;                               // chunked render passes have no workgroup
      S.fail_reason = DSR_FAIL_RENDER_FEW;              // for a ray-less object to fail it in)
    }
    if (S.lite_redo) {                                  // an audit caught a misclassification:
      S.lite_margin = 1e30f;                            // every sample exact from now on
    } else if (S.iters_done == 0) {
      S.lite_margin = P.lite_margin0;
    } else {
      const float m = fmaxf(P.lite_floor, P.lite_safety * S.lite_err);
      S.lite_margin = (m <= 0.1f) ? m : 1e30f;          // beyond: every sample exact
    }
#ifdef DSR_EXP_PROV
    prov_state(0, S.iters_done, desc[o].ray_off, prov_sum(S.T, S.depths, M));
#endif
  }
  __syncthreads();
  const ObjDesc d = desc[o];
  const float bg = S.bg_depth;
  for (int r = d.n_fg + tid; r < d.n_rays; r += blockDim.x) dobs[d.ray_off + r] = bg;
}

// ------------------------------------------------------------------------------------
// ray samples -> object frame -> |x| < 1 (loss.py:71-82)
// ------------------------------------------------------------------------------------
constexpr int SAMPLE_THREADS = 1024;

__device__ __forceinline__ float3 ray_sample(const float* __restrict__ rays, const ObjState& S,
                                             int ray, int j) {
  const float d = S.depths[j];
  const float cx = rays[ray * 3 + 0] * d, cy = rays[ray * 3 + 1] * d, cz = rays[ray * 3 + 2] * d;
  return xform(S.T, cx, cy, cz);
}
// The same sample from an LDS copy of the object's depths and pose (SampleLds) and the ray
// held in registers: the per-sample loop does no global loads.
struct SampleLds {
  float T[12];
  float depths[MAXM];
};
__device__ __forceinline__ void stage_samples(SampleLds& L, const ObjState& S, int M, int tid) {
  if (tid < 12) L.T[tid] = S.T[tid];
  if (tid < M) L.depths[tid] = S.depths[tid];
}
__device__ __forceinline__ float3 ray_sample(const float3 r, const SampleLds& L, int j) {
  const float d = L.depths[j];
  return xform(L.T, r.x * d, r.y * d, r.z * d);
}

// ------------------------------------------------------------------------------------
// Render passes: the ray samples of loss.py:71-82, emitted in render passes with early
// ray termination.  Pass [ra, rb) emits, for every ray not yet flagged dead, its
// in-ball samples of in-ball rank ra..rb-1 (rank = position among the ray's in-ball
// samples, depth order).  `dense` is NaN-filled before the first pass (out-of-ball samples
// stay NaN; samples behind a terminated ray are never read).  A ray is flagged dead by the fwd kernel when one of its samples
// decodes to sdf <= -th: its occupancy is then exactly 1 (0.5 - (-th)/(2 th), loss_utils.py
// :46-47), the cumulative transmittance exactly 0 from there on (loss.py:111), so every
// later sample of the ray enters d_u, var_u and de_do (loss.py:112-132) multiplied by an
// exact zero, and its de_do = 0 fails the 1e-2 filter (:135): decoding it cannot change
// any output, and k_render sees it only behind T == 0.  Results are bit-identical to
// decoding every in-ball sample; the first pass also marks the out-of-ball samples (NaN)
// and counts n_valid (loss.py:82-88) over ALL in-ball samples.
// One thread per ray, (ray, depth)-ordered output (k_sample_scan / _count / _emit below).
// ------------------------------------------------------------------------------------
// Ray chunks: k_refine_* and k_render_* run one workgroup per RENDER_RAYS rays of an object
// (table built once per batch), so an object's rays are processed side by side.
constexpr int RENDER_RAYS = 128;

struct RenderChunk {
  int obj;        // object index within the launch
  int ray0;       // first ray of the chunk (object-local)
  int first;      // launch-table index of the object's first chunk
  int n;          // chunks of the object
};

__device__ __forceinline__ int wave_incl_scan(int v, int lane) {
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int t = __shfl_up(v, o);
    if (lane >= o) v += t;
  }
  return v;
}

// One object's chunk counts cnt[stride * c], c in [c0, c0 + n), by one thread, 8 loads in flight.
__device__ __forceinline__ int object_chunk_sum(const int* __restrict__ cnt, int stride, int c0, int n) {
  int t = 0;
  for (int k = 0; k < n; k += 8) {
    int v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = (k + u < n) ? cnt[(size_t)stride * (c0 + k + u)] : 0;
#pragma unroll
    for (int u = 0; u < 8; ++u) t += v[u];
  }
  return t;
}

// ------------------------------------------------------------------------------------
// tile tables (single workgroup)
// ------------------------------------------------------------------------------------
// Tile tables (one block of 1024 threads): a block-wide exclusive scan of the per-object tile
// counts gives every object its first tile; then the whole block writes the tiles, thread t
// taking tiles t, t + 1024, ... of the chunk and finding its object by a binary search over
// the chunk's first-tile offsets in LDS (one thread per object writing all of that object's
// tiles was a serial loop of ~250 stores for one KITTI object's render pass, ~10 us).
// Object order, then tile order within an object — the table the serial loop would build.
constexpr int TILE_SCAN_THREADS = 1024;
template <class Count, class Emit>
__device__ __forceinline__ int tile_scan(int n_obj, int base, Count count, Emit emit) {
  __shared__ int wsum[16];
  __shared__ int carry;
  __shared__ int first_s[TILE_SCAN_THREADS + 1];   // chunk-relative first tile per object, + total
  __shared__ int n_s[TILE_SCAN_THREADS];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, nw = blockDim.x >> 6;
  if (tid == 0) carry = base;
  __syncthreads();
  for (int o0 = 0; o0 < n_obj; o0 += blockDim.x) {
    const int o = o0 + tid;
    const int m = min((int)blockDim.x, n_obj - o0);   // objects in this chunk
    int n = 0, nt = 0;
    if (o < n_obj) count(o, n, nt);
    const int inc = wave_incl_scan(nt, lane);
    if (lane == 63) wsum[wv] = inc;
    __syncthreads();
    if (wv == 0) {
      int v = lane < nw ? wsum[lane] : 0;
      v = wave_incl_scan(v, lane);
      if (lane < nw) wsum[lane] = v;
    }
    __syncthreads();
    if (tid < m) {
      first_s[tid] = (wv ? wsum[wv - 1] : 0) + inc - nt;
      n_s[tid] = n;
    }
    if (tid == 0) first_s[m] = wsum[nw - 1];
    __syncthreads();
    const int c0 = carry, ct = first_s[m];
    for (int t = tid; t < ct; t += blockDim.x) {
      int lo = 0, hi = m - 1;                 // last object whose first tile is <= t
      while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (first_s[mid] <= t) lo = mid; else hi = mid - 1;
      }
      emit(c0 + t, o0 + lo, t - first_s[lo], n_s[lo]);
    }
    __syncthreads();
    if (tid == 0) carry += ct;
    __syncthreads();
  }
  return carry;
}

// with_pts (exact pass, kept masks): each object's sample tiles, then its surface-point
// tiles (term 3, the same 64-point groups as the Jacobian's sdf tiles).  `count(o)` gives an
// object's samples, or -1 for an object that gets no tile.
template <class Count>
__device__ __forceinline__ void build_tiles_fwd(int n_obj, const ObjDesc* __restrict__ desc, Count count,
                                                Tile* __restrict__ tiles, int* __restrict__ n_tiles, int tsize,
                                                int with_pts) {
  const int total = tile_scan(
      n_obj, 0,
      [&](int o, int& n, int& nt) {
        const int c = count(o);
        n = max(c, 0);
        nt = (n + tsize - 1) / tsize;
        if (with_pts && c >= 0) nt += (desc[o].n_pts + TILE - 1) / TILE;
      },
      [&](int idx, int o, int i, int n) {
        Tile t;
        const int nb = (n + tsize - 1) / tsize;
        t.obj = o;
        if (i < nb) {
          t.term = 0; t.start = i * tsize;
          t.count = min(tsize, n - i * tsize);
        } else {
          t.term = 3; t.start = (i - nb) * TILE;
          t.count = min(TILE, desc[o].n_pts - t.start);
        }
        tiles[idx] = t;
      });
  if (threadIdx.x == 0) *n_tiles = total;
}

__global__ void k_tiles_fwd(int n_obj, const ObjDesc* __restrict__ desc, const ObjState* __restrict__ st,
                            Tile* __restrict__ tiles, int* __restrict__ n_tiles, int tsize, int with_pts) {
  build_tiles_fwd(
      n_obj, desc, [&](int o) { return st[o].status == ST_RUNNING ? st[o].n_emit : -1; }, tiles, n_tiles,
      tsize, with_pts);
}

// Every object's sdf tiles (forward + backward) first, then every render tile (backward
// only, kept masks): the persistent grid's blocks then run tiles of one kind together, so
// the layers they stream stay in step (L2-resident weights).  Tile outputs go to slots
// derived from the tile itself (jac_tail), so the order changes no result.  `k_of(o)`: the
// object's render points K.
template <class KOf>
__device__ __forceinline__ void build_tiles_jac(int n_obj, const ObjDesc* __restrict__ desc, ObjState* st, KOf k_of,
                                                Tile* __restrict__ tiles, int* __restrict__ n_tiles) {
  int total = 0;
  for (int term = 0; term < 2; ++term)
    total = tile_scan(
        n_obj, total,
        [&](int o, int& n, int& nt) {
          ObjState& S = st[o];
          n = (S.status == ST_RUNNING) ? (term == 0 ? desc[o].n_pts : k_of(o)) : 0;
          nt = (n + TILE - 1) / TILE;
          if (term == 0) S.n_sdf_tiles = nt;
          else S.n_ren_tiles = nt;
        },
        [&](int idx, int o, int i, int n) {
          Tile t;
          t.obj = o; t.term = term; t.start = i * TILE;
          t.count = min(TILE, n - i * TILE);
          tiles[idx] = t;
        });
  if (threadIdx.x == 0) *n_tiles = total;
}

__global__ void k_tiles_jac(int n_obj, const ObjDesc* __restrict__ desc, ObjState* st,
                            Tile* __restrict__ tiles, int* __restrict__ n_tiles) {
  build_tiles_jac(n_obj, desc, st, [&](int o) { return st[o].k; }, tiles, n_tiles);
}

// The same tables built by one extra workgroup of the emit / gather kernels of the chunked
// (one-group) path, from the per-chunk counts the previous launch left — the counts the
// emitting workgroups turn into S.n_emit / S.n_refine / S.k meanwhile — so no workgroup waits
// on another and the separate table launch (~4 us + its gap) goes.  `och[o]` = the object's
// first chunk and chunk count.  First pass: an object with fewer than 10 in-ball samples gets
// no tile (the emitting workgroups fail it, loss.py:86-88), as k_tiles_fwd would see it.
struct ChunkTiles {
  const int2* och;   // nullptr: no extra workgroup (the kernel's grid is the chunks)
  Tile* tiles;
  int* n_tiles;
  int n_obj, tsize, with_pts;
};
__device__ __forceinline__ void chunk_tiles_fwd(const ChunkTiles& T, const ObjDesc* __restrict__ desc,
                                                const ObjState* __restrict__ st, const int* __restrict__ cnt,
                                                int stride, const int* __restrict__ nin) {
  build_tiles_fwd(
      T.n_obj, desc,
      [&](int o) {
        const int2 oc = T.och[o];
        if (st[o].status != ST_RUNNING) return -1;
        if (nin && object_chunk_sum(nin, stride, oc.x, oc.y) < 10) return -1;
        return object_chunk_sum(cnt, stride, oc.x, oc.y);
      },
      T.tiles, T.n_tiles, T.tsize, T.with_pts);
}

// Chunked render passes (one thread per ray, one workgroup per RENDER_RAYS rays of an object,
// the render chunk table): a pass is a count kernel — k_sample_scan for the first pass, which
// also records each ray's in-ball run (loss.py:82) and clears its dead flag, k_sample_count for
// later passes — then k_sample_emit, which places every chunk at the sum of the earlier chunks'
// counts: the (ray, depth)-ordered list k_sample_pass's one workgroup per object builds, spread
// over the CUs (one KITTI object: 18 workgroups instead of one).  Per ray the count kernel leaves
// rwin = cnt | (j0 + 1) << 8 (j0 = the ray's first in-ball sample, -1 when its in-ball set is not
// one run: k_sample_emit then walks the ray); per chunk sc[2c] = samples emitted, sc[2c + 1] =
// in-ball samples (first pass: n_valid, loss.py:82-88).  Launched per object group with the
// group's own descriptor / state slices and chunk table (RenderChunk.obj is group-relative), so
// no workgroup touches another group's rays.
// (no packed-FP32 VALU ops in the kernels that form ray samples — k_sample_scan / _count /
// _emit / _pass and k_refine_emit: DESIGN.md §3.9 — under concurrent decoder kernels the
// SLP-paired v_pk_mul_f32 of the scan loop's first trip returned wrong products in one quarter-wave)
__device__ __forceinline__ void chunk_sums(int a, int b, int* __restrict__ out) {
  __shared__ int ws[2][RENDER_RAYS / 64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
  for (int k = 32; k > 0; k >>= 1) {
    a += __shfl_xor(a, k);
    b += __shfl_xor(b, k);
  }
  if (lane == 0) { ws[0][wv] = a; ws[1][wv] = b; }
  __syncthreads();
  if (threadIdx.x == 0) {
    int x = 0, y = 0;
    for (int k = 0; k < RENDER_RAYS / 64; ++k) { x += ws[0][k]; y += ws[1][k]; }
    out[0] = x;
    out[1] = y;
  }
}

// v[stride * c] summed over chunks c in [c0, c1) by the whole block (call it uniformly): the
// loads in parallel, one latency, where a serial walk over an object's earlier chunks waited
// once per chunk (up to ~1 us each, ~18 chunks for a KITTI object).  Integer sums: any order.
__device__ __forceinline__ int block_chunk_sum(const int* __restrict__ v, int stride, int c0, int c1) {
  __shared__ int ws[16];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
  int x = 0;
  for (int c = c0 + (int)threadIdx.x; c < c1; c += blockDim.x) x += v[(size_t)stride * c];
#pragma unroll
  for (int k = 32; k > 0; k >>= 1) x += __shfl_xor(x, k);
  if (lane == 0) ws[wv] = x;
  __syncthreads();
  int t = 0;
  for (int k = 0; k < nw; ++k) t += ws[k];
  __syncthreads();                       // (ws reusable by the next call)
  return t;
}

// The in-ball samples of ranks [ra, rb) of a ray whose in-ball set is not one run (rank =
// position among the ray's in-ball samples, depth order): their number, and the ray's in-ball
// total when the walk is not cut at rb.
__device__ __forceinline__ int walk_count(const float3 rv, const SampleLds& L, int M, int ra, int rb,
                                          bool cut, int& nin) {
  int rank = 0, cnt = 0;
  for (int j = 0; j < M; ++j) {
    const float3 x = ray_sample(rv, L, j);
    const float nrm = sqrtf((x.x * x.x + x.y * x.y) + x.z * x.z);   // torch.norm(.., dim=-1)
    if (!(nrm < 1.0f)) continue;                                      // loss.py:82
    if (rank >= ra && rank < rb) ++cnt;
    ++rank;
    if (cut && rank >= rb) break;
  }
  nin = rank;
  return cnt;
}

__global__ __launch_bounds__(RENDER_RAYS) DSR_NO_PK_F32 void k_sample_scan(const RenderChunk* __restrict__ chunks,
                                                             const ObjDesc* __restrict__ desc,
                                                             const ObjState* __restrict__ st,
                                                             const float* __restrict__ rays_all, int M, int rb,
                                                             int* __restrict__ dead, int* __restrict__ rinfo,
                                                             int* __restrict__ rwin, int* __restrict__ sc,
                                                             float* __restrict__ dense) {
  const RenderChunk ch = chunks[blockIdx.x];
  const ObjState& S = st[ch.obj];
  if (S.status != ST_RUNNING) return;
  const ObjDesc d = desc[ch.obj];
  __shared__ SampleLds L;
  stage_samples(L, S, M, threadIdx.x);
  {   // the chunk's rows of the sample values: NaN = out of the ball (loss.py:82; the passes'
      // decodes overwrite the in-ball samples they reach)
    const int nr = max(0, min(RENDER_RAYS, d.n_rays - ch.ray0));
    float* row = dense + d.cand_off + (size_t)ch.ray0 * M;
    for (int e = threadIdx.x; e < nr * M; e += RENDER_RAYS) row[e] = __builtin_nanf("");
  }
  __syncthreads();
#ifdef DSR_EXP_PROV
  if (threadIdx.x == 0) prov_state(1, S.iters_done, d.ray_off + ch.ray0, prov_sum(L.T, L.depths, M));
#endif
  const int ray = ch.ray0 + threadIdx.x;
  int cnt = 0, rank = 0;
  if (ray < d.n_rays) {
    const float* rays = rays_all + (size_t)d.ray_off * 3;
    const float3 rv = make_float3(rays[ray * 3 + 0], rays[ray * 3 + 1], rays[ray * 3 + 2]);
    dead_put(dead + d.ray_off + ray, 0);
#ifdef DSR_EXP_PROV
    prov_clear(S.iters_done, d.ray_off + ray);
#endif
    int jf = -1, jl = -1;
    for (int j = 0; j < M; ++j) {
      const float3 x = ray_sample(rv, L, j);
      const float nrm = sqrtf((x.x * x.x + x.y * x.y) + x.z * x.z);   // torch.norm(.., dim=-1)
      if (!(nrm < 1.0f)) continue;
      if (jf < 0) jf = j;
      jl = j;
      ++rank;
    }
    // the in-ball set of a ray is one run of samples unless rounding makes |x| < 1 flicker
    // near a tangent point; such rays are walked again in every pass
    const int info = rank == 0 ? 0 : (jl - jf + 1 == rank ? (jf | (rank << 8)) : -1);
    rinfo[d.ray_off + ray] = info;
    cnt = min(rank, rb);
    const int j0 = info >= 0 ? (info & 255) : -1;
    rwin[d.ray_off + ray] = cnt | ((j0 + 1) << 8);
#ifdef DSR_EXP_PROV
    prov_rinfo(0, S.iters_done, d.ray_off + ray, info);
    prov_alive(S.iters_done, 0, d.ray_off + ray, cnt + 1);
    prov_emit(S.iters_done, 0, d.ray_off + ray, cnt > 0 ? (j0 >= 0 ? j0 : -2) : -1);
#endif
  }
  chunk_sums(cnt, rank, sc + 2 * blockIdx.x);
}

// later passes [ra, rb): the rays not flagged dead by the earlier passes' decodes
__global__ __launch_bounds__(RENDER_RAYS) DSR_NO_PK_F32 void k_sample_count(const RenderChunk* __restrict__ chunks,
                                                              const ObjDesc* __restrict__ desc,
                                                              const ObjState* __restrict__ st,
                                                              const float* __restrict__ rays_all, int M, int ra,
                                                              int rb, int* __restrict__ dead,
                                                              const int* __restrict__ rinfo,
                                                              int* __restrict__ rwin, int* __restrict__ sc) {
  const RenderChunk ch = chunks[blockIdx.x];
  const ObjState& S = st[ch.obj];
  if (S.status != ST_RUNNING) return;
  const ObjDesc d = desc[ch.obj];
  __shared__ SampleLds L;
  stage_samples(L, S, M, threadIdx.x);
  __syncthreads();
  const int ray = ch.ray0 + threadIdx.x;
  int cnt = 0;
  if (ray < d.n_rays) {
    const bool alive = dead_get(dead + d.ray_off + ray) == 0;
    int j0 = -1;
    if (alive) {
      const int info = rinfo[d.ray_off + ray];
      if (info >= 0) {
        j0 = info & 255;
        cnt = max(0, min(rb, info >> 8) - ra);
      } else {
        const float* rp = rays_all + (size_t)(d.ray_off + ray) * 3;
        int nin;
        cnt = walk_count(make_float3(rp[0], rp[1], rp[2]), L, M, ra, rb, true, nin);
      }
    }
    rwin[d.ray_off + ray] = cnt | ((j0 + 1) << 8);
#ifdef DSR_EXP_PROV
    prov_alive(S.iters_done, ra, d.ray_off + ray, alive ? cnt + 1 : -1);
    prov_emit(S.iters_done, ra, d.ray_off + ray, cnt > 0 ? (j0 >= 0 ? j0 + ra : -2) : -1);
#endif
  }
  chunk_sums(cnt, 0, sc + 2 * blockIdx.x);
}

__global__ __launch_bounds__(RENDER_RAYS) DSR_NO_PK_F32 void k_sample_emit(const RenderChunk* __restrict__ chunks,
                                                             const ObjDesc* __restrict__ desc, ObjState* st,
                                                             const float* __restrict__ rays_all, int M, int ra,
                                                             int rb, float4* __restrict__ cand,
                                                             const int* __restrict__ rwin,
                                                             const int* __restrict__ sc, ChunkTiles T) {
  if (T.och && (int)blockIdx.x == (int)gridDim.x - 1) {   // the extra workgroup: the pass's tile table
    chunk_tiles_fwd(T, desc, st, sc, 2, ra == 0 ? sc + 1 : nullptr);
    return;
  }
  const RenderChunk ch = chunks[blockIdx.x];
  ObjState& S = st[ch.obj];
  if (S.status != ST_RUNNING) return;
  const ObjDesc d = desc[ch.obj];
  __shared__ int wsum[RENDER_RAYS / 64];
  __shared__ SampleLds L;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  stage_samples(L, S, M, tid);
  const bool last = (int)blockIdx.x == ch.first + ch.n - 1;   // the object's last chunk: its totals
  const int base = block_chunk_sum(sc, 2, ch.first, blockIdx.x);
  const int nin = (last && ra == 0) ? block_chunk_sum(sc + 1, 2, ch.first, blockIdx.x + 1) : 0;
  const int ray = ch.ray0 + tid;
  int cnt = 0, j0 = -1;
  float3 rv = make_float3(0.f, 0.f, 0.f);
  if (ray < d.n_rays) {
    const int w = rwin[d.ray_off + ray];
    cnt = w & 255;
    j0 = (w >> 8) - 1;
    if (cnt > 0) {
      const float* rp = rays_all + (size_t)(d.ray_off + ray) * 3;
      rv = make_float3(rp[0], rp[1], rp[2]);
    }
  }
  const int inc = wave_incl_scan(cnt, lane);
  if (lane == 63) wsum[wv] = inc;
  __syncthreads();
  int off = d.cand_off + base + inc - cnt;
  for (int k = 0; k < wv; ++k) off += wsum[k];
  if (cnt > 0 && j0 >= 0) {
    for (int k = ra; k < ra + cnt; ++k) {
      const float3 x = ray_sample(rv, L, j0 + k);
      cand[off++] = make_float4(x.x, x.y, x.z, __int_as_float(ray * M + j0 + k));
    }
  } else if (cnt > 0) {
    int rank = 0;
    for (int j = 0; j < M && rank < rb; ++j) {
      const float3 x = ray_sample(rv, L, j);
      const float nrm = sqrtf((x.x * x.x + x.y * x.y) + x.z * x.z);
      if (!(nrm < 1.0f)) continue;
      if (rank >= ra) cand[off++] = make_float4(x.x, x.y, x.z, __int_as_float(ray * M + j));
      ++rank;
    }
  }
  if (tid == 0 && last) {
    int t = base;
    for (int k = 0; k < RENDER_RAYS / 64; ++k) t += wsum[k];
    S.n_emit = t;
    S.n_eval += t;
    if (ra == 0) {
      S.n_valid = nin;
      if (nin < 10) {                          // loss.py:86-88 -> optimizer.py:144-145
        S.status = ST_FAIL;
        S.fail_reason = DSR_FAIL_RENDER_FEW;
      }
    }
  }
}

// ------------------------------------------------------------------------------------
// k_sample_pass: the same pass in one 1024-thread workgroup per object walking its rays in
// rounds — the multi-group batches' form (measured equal to the chunked one there, DESIGN.md
// §3.8) and, under DSR_PRESCAN=0, the schedule tests' second implementation for one group; the
// first pass included: it clears the dead flags, records the runs and counts n_valid itself.
// k_tiles_fwd then builds the pass's tile table from S.n_emit.
// ------------------------------------------------------------------------------------
__global__ __launch_bounds__(SAMPLE_THREADS) DSR_NO_PK_F32 void k_sample_pass(int n_obj, const ObjDesc* __restrict__ desc,
                                                                ObjState* st, const float* __restrict__ rays_all,
                                                                int M, int ra, int rb, float4* __restrict__ cand,
                                                                int* __restrict__ dead, int* __restrict__ rinfo) {
  const int o = blockIdx.x;
  ObjState& S = st[o];
  if (S.status != ST_RUNNING) return;
  const ObjDesc d = desc[o];
  const float* rays = rays_all + (size_t)d.ray_off * 3;
  const bool first = ra == 0;
  __shared__ int wsum[SAMPLE_THREADS / 64];
  __shared__ int wnin[SAMPLE_THREADS / 64];
  __shared__ int base_s, nin_s;
  __shared__ SampleLds L;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  if (tid == 0) { base_s = 0; nin_s = 0; }
  stage_samples(L, S, M, tid);
  __syncthreads();
  for (int r0 = 0; r0 < d.n_rays; r0 += SAMPLE_THREADS) {
    const int ray = r0 + tid;
    int cnt = 0, nin = 0;
    int j0 = -1;                  // later passes: the ray's in-ball samples are j0 .. j0+nin-1
    float3 rv = make_float3(0.f, 0.f, 0.f);
    if (ray < d.n_rays) {
      rv = make_float3(rays[ray * 3 + 0], rays[ray * 3 + 1], rays[ray * 3 + 2]);
      if (first) dead_put(dead + d.ray_off + ray, 0);
      const bool alive = first || dead_get(dead + d.ray_off + ray) == 0;
      if (alive && !first) {
        const int info = rinfo[d.ray_off + ray];
        if (info >= 0) {          // contiguous in-ball run: the window directly
          j0 = info & 255;
          nin = info >> 8;
          cnt = max(0, min(rb, nin) - ra);
        }
      }
      if (alive && j0 < 0) {
        if (first) {
          int rank = 0, jf = -1, jl = -1;
          for (int j = 0; j < M; ++j) {
            const float3 x = ray_sample(rv, L, j);
            const float nrm = sqrtf((x.x * x.x + x.y * x.y) + x.z * x.z);   // torch.norm(.., dim=-1)
            if (!(nrm < 1.0f)) continue;   // loss.py:82 (out of ball: NaN, dense pre-filled)
            if (jf < 0) jf = j;
            jl = j;
            if (rank < rb) ++cnt;
            ++rank;
          }
          nin = rank;
          rinfo[d.ray_off + ray] = rank == 0 ? 0 : (jl - jf + 1 == rank ? (jf | (rank << 8)) : -1);
        } else {
          cnt = walk_count(rv, L, M, ra, rb, true, nin);
        }
      }
    }
    const int inc = wave_incl_scan(cnt, lane);
    int nin_w = nin;
#pragma unroll
    for (int k = 32; k > 0; k >>= 1) nin_w += __shfl_xor(nin_w, k);
    if (lane == 63) wsum[wv] = inc;
    if (lane == 0) wnin[wv] = nin_w;
    __syncthreads();
    int off = base_s + inc - cnt;
    for (int k = 0; k < wv; ++k) off += wsum[k];
    if (cnt > 0 && j0 >= 0) {
      for (int k = ra; k < ra + cnt; ++k) {
        const float3 x = ray_sample(rv, L, j0 + k);
        cand[d.cand_off + off++] = make_float4(x.x, x.y, x.z, __int_as_float(ray * M + j0 + k));
      }
    } else if (cnt > 0) {
      int rank = 0;
      for (int j = 0; j < M && rank < rb; ++j) {
        const float3 x = ray_sample(rv, L, j);
        const float nrm = sqrtf((x.x * x.x + x.y * x.y) + x.z * x.z);
        if (!(nrm < 1.0f)) continue;
        if (rank >= ra) cand[d.cand_off + off++] = make_float4(x.x, x.y, x.z, __int_as_float(ray * M + j));
        ++rank;
      }
    }
    __syncthreads();
    if (tid == 0) {
      int t = 0, u = 0;
      for (int k = 0; k < SAMPLE_THREADS / 64; ++k) { t += wsum[k]; u += wnin[k]; }
      base_s += t;
      nin_s += u;
    }
    __syncthreads();
  }
  if (tid == 0) {
    S.n_emit = base_s;
    S.n_eval += base_s;
    if (first) {
      S.n_valid = nin_s;
      if (nin_s < 10) {                        // loss.py:86-88 -> optimizer.py:144-145
        S.status = ST_FAIL;
        S.fail_reason = DSR_FAIL_RENDER_FEW;
      }
    }
  }
}

// ------------------------------------------------------------------------------------
// k_refine_scan + k_refine_emit: the samples the lite pass left in the +-(th + margin) band
// (dsr_mlp_lite.hpp), (ray, depth)-ordered into cand for the exact split-fp16 pass; the
// scan clears the flags it consumes.  One thread per ray, one workgroup per chunk of
// RENDER_RAYS rays (the render chunk table): the scan records each ray's refined and
// audited sample bits and the chunk's count; the emit places every chunk at the sum of the
// earlier chunks' counts — the list one sequential pass over the rays would build.
// A ray's scan stops at its first certainly-full sample (an unflagged lite value
// <= -th - margin, the criterion that set `dead`): its exact sdf is <= -th, so the
// transmittance is exactly 0 behind it and every later sample enters d_u, de_do and K
// (loss.py:111-135) multiplied by that zero (the early-termination argument, DESIGN
// §3.3) — band samples there need no exact value.  Every sample in front of it was
// decoded by this iteration's passes (in-ball rank = depth order), and out-of-ball
// samples hold NaN, so the scan reads only this iteration's values.  `dense` == nullptr
// refines every flagged sample (DSR_REFINE_ALL=1).
// ------------------------------------------------------------------------------------
constexpr int REFINE_SCAN_THREADS = 256;   // 4 waves x 32 rays of a chunk: one round of loads each
__global__ __launch_bounds__(REFINE_SCAN_THREADS) void k_refine_scan(const RenderChunk* __restrict__ chunks,
                                                             const ObjDesc* __restrict__ desc, ObjState* st,
                                                             int M, unsigned char* __restrict__ refine,
                                                             const float* __restrict__ dense, float nth,
                                                             uint64_t* __restrict__ rbits_g,
                                                             uint64_t* __restrict__ abits_g, int* __restrict__ ccnt,
                                                             int* __restrict__ slotmap) {
  const RenderChunk ch = chunks[blockIdx.x];
  ObjState& S = st[ch.obj];
  if (S.status != ST_RUNNING) return;
  const ObjDesc d = desc[ch.obj];
  constexpr int NW = REFINE_SCAN_THREADS / 64, RPW = RENDER_RAYS / NW;   // waves, rays per wave
  __shared__ uint64_t rbits[RENDER_RAYS], abits[RENDER_RAYS];
  __shared__ int wsum[2][NW];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const float full = nth - S.lite_margin;
  // Each wave scans its RPW rays one at a time, lane j on sample j (coalesced flag / value
  // loads — all RPW rays' in flight at once — and ballots): refined = the flagged samples in
  // front of the first unflagged sample that is certainly full, or up to and including it when
  // it is an audited full sample (flag 3); every flag is cleared.  Flags 2/3 (audit, lite_flag)
  // ride along in bit 30 of the candidate's index so the exact pass can check their class.
  {
    unsigned char fv[RPW];
    float yv[RPW];
#pragma unroll
    for (int u = 0; u < RPW; ++u) {
      const int rr = ch.ray0 + RPW * wv + u;
      const bool in = rr < d.n_rays && lane < M;
      const size_t e = d.cand_off + (size_t)rr * M + lane;
      fv[u] = in ? refine[e] : 0;
      yv[u] = (in && dense) ? dense[e] : __builtin_nanf("");
    }
#pragma unroll
    for (int u = 0; u < RPW; ++u) {
      const int rr = ch.ray0 + RPW * wv + u;
      const uint64_t fb = __ballot(fv[u] != 0);
      const uint64_t ub = __ballot((fv[u] == 0 || fv[u] == 3) && yv[u] <= full);
      const uint64_t tb = __ballot(fv[u] == 3), ab = __ballot(fv[u] >= 2);
      uint64_t b = fb;
      if (ub) {
        const int stop = __builtin_ctzll(ub);
        b = fb & (((1ull << stop) - 1) | (tb & (1ull << stop)));
      }
      if (rr < d.n_rays && lane < M) {
        refine[d.cand_off + (size_t)rr * M + lane] = 0;
        if (slotmap) slotmap[d.cand_off + (size_t)rr * M + lane] = -1;   // k_refine_emit sets the refined
      }
      if (lane == u) {
        rbits[RPW * wv + u] = b;
        abits[RPW * wv + u] = b & ab;
      }
    }
  }
  __syncthreads();
  int cnt = 0, n_audit = 0;
  if (tid < RENDER_RAYS) {
    const uint64_t bits = rbits[tid], aud = abits[tid];
    const int ray = ch.ray0 + tid;
    if (ray < d.n_rays) {
      rbits_g[d.ray_off + ray] = bits;
      abits_g[d.ray_off + ray] = aud;
    }
    cnt = __popcll(bits);
    n_audit = __popcll(aud);
  }
#pragma unroll
  for (int k = 32; k > 0; k >>= 1) {
    cnt += __shfl_xor(cnt, k);
    n_audit += __shfl_xor(n_audit, k);
  }
  if (lane == 0) { wsum[0][wv] = cnt; wsum[1][wv] = n_audit; }
  __syncthreads();
  if (tid == 0) {
    int t = 0, a = 0;
    for (int k = 0; k < NW; ++k) { t += wsum[0][k]; a += wsum[1][k]; }
    ccnt[blockIdx.x] = t;
    if (a) atomicAdd(&S.n_audit, a);           // one atomic per chunk
  }
}

__global__ __launch_bounds__(RENDER_RAYS) DSR_NO_PK_F32 void k_refine_emit(const RenderChunk* __restrict__ chunks,
                                                             const ObjDesc* __restrict__ desc, ObjState* st,
                                                             const float* __restrict__ rays_all, int M,
                                                             float4* __restrict__ cand, int* __restrict__ slotmap,
                                                             const uint64_t* __restrict__ rbits_g,
                                                             const uint64_t* __restrict__ abits_g,
                                                             const int* __restrict__ ccnt, ChunkTiles T) {
  if (T.och && (int)blockIdx.x == (int)gridDim.x - 1) {   // the extra workgroup: the exact pass's tiles
    chunk_tiles_fwd(T, desc, st, ccnt, 1, nullptr);
    return;
  }
  const RenderChunk ch = chunks[blockIdx.x];
  ObjState& S = st[ch.obj];
  if (S.status != ST_RUNNING) return;
  const ObjDesc d = desc[ch.obj];
  __shared__ int wsum[RENDER_RAYS / 64];
  __shared__ SampleLds L;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  stage_samples(L, S, M, tid);
  const int base = block_chunk_sum(ccnt, 1, ch.first, blockIdx.x);
  const int ray = ch.ray0 + tid;
  uint64_t bits = 0, aud = 0;
  float3 rv = make_float3(0.f, 0.f, 0.f);
  if (ray < d.n_rays) {
    bits = rbits_g[d.ray_off + ray];
    aud = abits_g[d.ray_off + ray];
    const float* rp = rays_all + (size_t)(d.ray_off + ray) * 3;
    rv = make_float3(rp[0], rp[1], rp[2]);
  }
  const int cnt = __popcll(bits);
  const int inc = wave_incl_scan(cnt, lane);
  if (lane == 63) wsum[wv] = inc;
  __syncthreads();
  int off = base + inc - cnt;
  for (int k = 0; k < wv; ++k) off += wsum[k];
  for (uint64_t m = bits; m; m &= m - 1) {
    const int j = __builtin_ctzll(m);
    const float3 x = ray_sample(rv, L, j);
    if (slotmap) slotmap[d.cand_off + ray * M + j] = off;
    const int tag = ((aud >> j) & 1) ? AUDIT_BIT : 0;
    cand[d.cand_off + off++] = make_float4(x.x, x.y, x.z, __int_as_float((ray * M + j) | tag));
  }
  if (tid == 0 && (int)blockIdx.x == ch.first + ch.n - 1) {
    int t = base;
    for (int k = 0; k < RENDER_RAYS / 64; ++k) t += wsum[k];
    S.n_emit = t;
    S.n_refine = t;
  }
}

// ------------------------------------------------------------------------------------
// k_mlp_fwd: decode_sdf over every in-ball ray sample (persistent, one tile per pass)
// ------------------------------------------------------------------------------------
struct FwdShared {
  float H[H_FLOATS];
  float xyz[TILE * 4];
  float red[NWAVE * TILE];
};

// V bit0: per-tile soft sync of each XCD's workgroups (L2 reuse of the layer weights)
// V bit1: B-fragment prefetch GEMM; V bit2: s_setprio around MFMA clusters
template <int V>
__device__ __forceinline__ void fwd_gemm(const float4* A, int T, const float* Hs, floatx4 (&acc)[4][4],
                                         int lane) {
  if constexpr ((V & 2) != 0) gemm_tile_pf<4, (V & 4) != 0>(A, T, Hs, acc, lane);
  else gemm_tile<4>(A, T, Hs, acc, lane);
}

template <int V>
__global__ __launch_bounds__(512) void k_mlp_fwd(DevDecoder D, const Tile* __restrict__ tiles,
                                                 const int* __restrict__ n_tiles,
                                                 const ObjDesc* __restrict__ desc,
                                                 const float4* __restrict__ cand,
                                                 const float* __restrict__ bias0f,
                                                 const float* __restrict__ bias4f,
                                                 float* __restrict__ dense,
                                                 unsigned* __restrict__ sync_ctr, ErtArgs E, MaskArgs) {
  __shared__ FwdShared sm;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nt = *n_tiles;
  const int rounds = (nt + gridDim.x - 1) / gridDim.x;
  for (int r = 0; r < rounds; ++r) {
    const int ti = blockIdx.x + r * gridDim.x;
    if constexpr ((V & 1) != 0) group_soft_sync(sync_ctr, r);
    if (ti >= nt) continue;
    const Tile tl = tiles[ti];
    const ObjDesc d = desc[tl.obj];
    const float4* src = cand + d.cand_off + tl.start;
    if (tid < TILE) {
      float4 v = (tid < tl.count) ? src[tid] : make_float4(0.f, 0.f, 0.f, 0.f);
      sm.xyz[tid * 4 + 0] = v.x; sm.xyz[tid * 4 + 1] = v.y;
      sm.xyz[tid * 4 + 2] = v.z; sm.xyz[tid * 4 + 3] = v.w;
    }
    __syncthreads();
    uint64_t mask;
    layer0_fwd(D, bias0f + tl.obj * HID, sm.xyz, sm.H, w, lane, mask);
    __syncthreads();
    floatx4 acc[4][4];
    for (int l = 1; l <= 6; ++l) {
      const int T = D.Kf[l] / 16;
      fwd_gemm<V>(D.Wf[l] + (size_t)(4 * w) * T * 64, T, sm.H, acc, lane);
      __syncthreads();
      epi_fwd(acc, (l == 4) ? bias4f + tl.obj * HID : D.bias[l], sm.H, sm.xyz, w, lane, mask, l == 3, D.l3);
      __syncthreads();
    }
    {
      const int T = D.Kf[7] / 16;
      fwd_gemm<V>(D.Wf[7] + (size_t)(4 * w) * T * 64, T, sm.H, acc, lane);
      epi_l7(acc, D, sm.red, w, lane, mask);
    }
    __syncthreads();
    if (tid < tl.count) {
      float s = sm.red[tid];
      for (int k = 1; k < NWAVE; ++k) s += sm.red[k * TILE + tid];
      const float y = tanhf(s + D.b8);
      const int idx = __float_as_int(sm.xyz[tid * 4 + 3]) & ~AUDIT_BIT;   // (audit tag: lite_flag)
      dense[d.cand_off + idx] = y;
      if (E.dead && y <= E.nth) dead_put(E.dead + d.ray_off + idx / E.M, 1);
    }
    __syncthreads();
  }
}

// ------------------------------------------------------------------------------------
// k_render_rays + k_render_gather: the per-ray occupancy scan of loss.py:97-150 and the
// ordered compaction of its K render points.  One thread per ray; an object's rays are
// split into chunks of RENDER_RAYS, one workgroup each (the table is built once per batch),
// so the ~5-20 chunks of an object run side by side instead of one workgroup walking the
// rays in rounds (a per-object latency that small batches cannot hide: 179 -> ~40 us per
// KITTI object).  Each chunk stages its rays' sdf rows in LDS twice (coalesced loads): the
// scan turns one copy into the transmittance rows, the other keeps the sdf values the
// de_do filter needs (no global re-reads inside the per-ray loops).  A chunk writes its
// render points, in (ray, depth) order, to a staging area at its own rays' sample range and
// its count; k_render_gather moves every chunk's points to the object's compacted K list
// at the sum of the earlier chunks' counts — the same list, in the same order, as one
// sequential pass over the rays.
// ------------------------------------------------------------------------------------

__device__ __forceinline__ float occupancy(float s, float nth, float th, float two_th) {
  // sdf_to_occupancy (loss_utils.py:40-48); NaN marks a sample outside the unit ball
  // (occ_values initialised to 0, loss.py:97-99)
  if (s != s) return 0.f;
  return 0.5f - fminf(fmaxf(s, nth), th) / two_th;
}

// LDS row pitch of the per-ray rows: odd, so the 64 lanes of a wave hit 64 different banks
__host__ __device__ constexpr int render_pitch(int M) { return (M + 1) | 1; }
__host__ __device__ constexpr size_t render_lds_bytes(int M) {
  return sizeof(float) * 2 * RENDER_RAYS * (size_t)render_pitch(M);
}

__global__ __launch_bounds__(RENDER_RAYS) void k_render_rays(const RenderChunk* __restrict__ chunks,
                                                             const ObjDesc* __restrict__ desc,
                                                             const ObjState* __restrict__ st,
                                                             const float* __restrict__ rays_all,
                                                             const float* __restrict__ dobs_all, GNParams P,
                                                             const float* __restrict__ dense,
                                                             float4* __restrict__ kst, float* __restrict__ rst,
                                                             int* __restrict__ sst, const int* __restrict__ slotmap,
                                                             int* __restrict__ ccnt) {
  const RenderChunk ch = chunks[blockIdx.x];
  const ObjState& S = st[ch.obj];
  if (S.status != ST_RUNNING) return;
  const ObjDesc d = desc[ch.obj];
  const int M = P.M, pitch = render_pitch(M);
  const float th = P.cut_off;
  const float nth = -th, two_th = 2.0f * th;
  const float do_ds = (float)(-1.0 / (2.0 * (double)th));
  extern __shared__ float render_lds[];
  float* T_s = render_lds;                       // transmittance rows (sdf until scanned)
  float* D_s = render_lds + RENDER_RAYS * pitch;  // sdf rows
  __shared__ float dep_s[MAXM];
  __shared__ int wsum[RENDER_RAYS / 64];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  if (tid < M) dep_s[tid] = S.depths[tid];
  const int nr = min(RENDER_RAYS, d.n_rays - ch.ray0);
  // this thread's ray: observed depth and direction, loaded now so their latency hides behind the
  // staging below (used after the scans)
  const int ray = ch.ray0 + tid;
  float dob = 0.f, rx = 0.f, ry = 0.f, rz = 0.f;
  if (tid < nr) {
    dob = dobs_all[d.ray_off + ray];
    const float* rp = rays_all + (size_t)(d.ray_off + ray) * 3;
    rx = rp[0]; ry = rp[1]; rz = rp[2];
  }
  {
    // The chunk's rows are one contiguous run of nr * M floats: read as 16-byte loads (a scalar
    // head up to the first aligned address, a scalar tail), all of a thread's loads in flight
    // before its LDS stores — one round of load latency (4-byte loads, 16 in flight, took 4)
    const float* src = dense + d.cand_off + (size_t)ch.ray0 * M;
    const int tot = nr * M;
    const int head = min(tot, (int)(((16 - ((uintptr_t)src & 15)) & 15) >> 2));
    const int n4 = (tot - head) >> 2, tail0 = head + 4 * n4;
    auto put = [&](int e, float v) {
      const int r = e / M, j = e - r * M;
      T_s[r * pitch + j] = v;
      D_s[r * pitch + j] = v;
    };
    constexpr int NV = (MAXM * RENDER_RAYS / 4 + RENDER_RAYS - 1) / RENDER_RAYS;
    const float4* s4 = reinterpret_cast<const float4*>(src + head);
    float4 v[NV];
#pragma unroll
    for (int u = 0; u < NV; ++u) {
      const int i = tid + u * RENDER_RAYS;
      v[u] = i < n4 ? s4[i] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    if (tid < head) put(tid, src[tid]);
    if (tid < tot - tail0) put(tail0 + tid, src[tail0 + tid]);
#pragma unroll
    for (int u = 0; u < NV; ++u) {
      const int i = tid + u * RENDER_RAYS;
      if (i < n4) {
        const int e = head + 4 * i;
        int r = e / M, j = e - r * M;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          T_s[r * pitch + j] = fetch4(v[u], k);
          D_s[r * pitch + j] = fetch4(v[u], k);
          if (++j == M) { j = 0; ++r; }
        }
      }
    }
  }
  __syncthreads();
  const float dmax = S.dmax, delta_d = S.delta_d;
  float* Tr = T_s + tid * pitch;
  float* Dr = D_s + tid * pitch;                  // sdf row; a kept sample's slot then holds its de_do
  int cnt = 0, jend = 0;
  float du = 0.f;
  uint64_t keep = 0;
  if (tid < nr) {
    // cumprod of (1 - o) (loss.py:111, sequential in fp32 like torch's), term
    // probabilities and rendered depth (:112-125).  The 51-term sum is accumulated in
    // fp64 and rounded once: torch's vectorised fp32 sum is within ~1 ulp of exact,
    // a sequential fp32 sum is not (d ~ 15 m, residual d_obs - d_u ~ 1 cm).
    // Once T == 0 (a sample with occupancy exactly 1) every later term probability,
    // transmittance and de_do is an exact 0: the scan stops there — the samples behind
    // were not decoded (early ray termination, k_sample_pass) and cannot matter.
    uint64_t grad = 0;
    float T = 1.f;
    double dud = 0.0;
    int j = 0;
    float s_next = Tr[0], d_next = dep_s[0];       // (next sample's LDS reads issued a step early)
    for (; j < M && T != 0.f; ++j) {
      const float s = s_next, dj = d_next;
      if (j + 1 < M) { s_next = Tr[j + 1]; d_next = dep_s[j + 1]; }
      const float ov = occupancy(s, nth, th, two_th);
      if (s > nth && s < th) grad |= 1ull << j;     // loss.py:101
      const float tp = ov * T;
      T = T * (1.f - ov);
      Tr[j] = T;
      dud += (double)(dj * tp);
    }
    jend = j;                                       // (samples l >= jend: transmittance 0)
    dud += (double)((1.1f * dmax) * T);            // background bin o=1, d=1.1*d_max
    du = (float)dud;
    // de_do of each band sample jj: the transmittance tail sum over l = jj .. jend-1 in fp64 (:131),
    // up to 4 band samples per sweep of the row, each sum still taken term by term from l = jj
    for (uint64_t m = grad; m;) {
      int jq[4];
      double acc[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        jq[q] = m ? __builtin_ctzll(m) : jend;
        m &= m - 1;
      }
      for (int l = jq[0]; l < jend; ++l) {
        const double t = (double)Tr[l];
#pragma unroll
        for (int q = 0; q < 4; ++q)
          if (l >= jq[q]) acc[q] += t;
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int jj = jq[q];
        if (jj >= jend) continue;
        const float dedo = (float)acc[q] / (1.f - occupancy(Dr[jj], nth, th, two_th));   // :131-132
        if (dedo > 1e-2f) { keep |= 1ull << jj; ++cnt; Dr[jj] = dedo; }                // :135
      }
    }
  }
  const int inc = wave_incl_scan(cnt, lane);
  if (lane == 63) wsum[wv] = inc;
  __syncthreads();
  int off = inc - cnt;
  for (int k = 0; k < wv; ++k) off += wsum[k];
  if (cnt > 0) {
    float res = dob - du;                           // :145
    res = res > 0.30f ? 0.30f : res;                // :147-148
    res = res < -0.30f ? -0.30f : res;
    const size_t base = (size_t)d.cand_off + (size_t)ch.ray0 * M;
    for (uint64_t m = keep; m; m &= m - 1) {
      const int jj = __builtin_ctzll(m);
      const float dedo = Dr[jj];
      const float deds = (dedo * delta_d) * do_ds;    // :142
      const float dj = dep_s[jj];
      const float3 x = xform(S.T, rx * dj, ry * dj, rz * dj);   // = ray_sample(rays, S, ray, jj)
      kst[base + off] = make_float4(x.x, x.y, x.z, deds);
      rst[base + off] = res;
      if (sst) sst[base + off] = slotmap[d.cand_off + ray * M + jj];
      ++off;
    }
  }
  if (tid == 0) {
    int t = 0;
    for (int k = 0; k < RENDER_RAYS / 64; ++k) t += wsum[k];
    ccnt[blockIdx.x] = t;
  }
}

// Every chunk's render points to the object's K list (offset = the earlier chunks' counts);
// the object's last chunk sets K.
__global__ __launch_bounds__(256) void k_render_gather(const RenderChunk* __restrict__ chunks,
                                                       const ObjDesc* __restrict__ desc, ObjState* st,
                                                       const int* __restrict__ ccnt, int M,
                                                       const float4* __restrict__ kst,
                                                       const float* __restrict__ rst,
                                                       const int* __restrict__ sst, float4* __restrict__ kpts,
                                                       float* __restrict__ kres, int* __restrict__ kslot,
                                                       ChunkTiles T) {
  if (T.och && (int)blockIdx.x == (int)gridDim.x - 1) {   // the extra workgroup: the Jacobian's tiles
    build_tiles_jac(
        T.n_obj, desc, st, [&](int o) { return object_chunk_sum(ccnt, 1, T.och[o].x, T.och[o].y); }, T.tiles,
        T.n_tiles);
    return;
  }
  const RenderChunk ch = chunks[blockIdx.x];
  ObjState& S = st[ch.obj];
  if (S.status != ST_RUNNING) return;
  const ObjDesc d = desc[ch.obj];
  const int off = block_chunk_sum(ccnt, 1, ch.first, blockIdx.x);
  const int n = ccnt[blockIdx.x];
  if (threadIdx.x == 0 && (int)blockIdx.x == ch.first + ch.n - 1) S.k = off + n;
  const size_t s0 = (size_t)d.cand_off + (size_t)ch.ray0 * M, d0 = (size_t)d.cand_off + off;
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    kpts[d0 + i] = kst[s0 + i];
    kres[d0 + i] = rst[s0 + i];
    if (kslot) kslot[d0 + i] = sst[s0 + i];
  }
}

// ------------------------------------------------------------------------------------
// k_mlp_jac: forward + analytic input Jacobian + per-tile normal-equation partials
// ------------------------------------------------------------------------------------
constexpr int JPITCH = 72;

// Tail shared by the fp32 and split-fp16 Jacobian kernels: raw output (dsr_sdf_eval), or
// J rows (loss.py:34-41 / :157-164) + Huber residuals + per-tile normal-equation partials.
__device__ __forceinline__ void jac_tail(const Tile& tl, const ObjDesc& d, const ObjState* __restrict__ st,
                                         const GNParams& P, float* __restrict__ slots,
                                         float* __restrict__ raw_out, float* __restrict__ res_out,
                                         const float* ys, const float* gin, const float* xyz, float* rs,
                                         float* Jbuf, int tid) {
    if (tl.term == 2) {            // raw query (dsr_sdf_eval): sdf + gradient out
      for (int e = tid; e < TILE * (IN + 1); e += 512) {
        const int p = e / (IN + 1), k = e - p * (IN + 1);
        if (p < tl.count)
          raw_out[(size_t)(tl.start + p) * (IN + 1) + k] = (k == 0) ? ys[p] : gin[p * GIN_PITCH + k - 1];
      }
      __syncthreads();
      return;
    }
    // ---- J rows (loss.py:34-41 / :157-164) into the freed H region
    float* J = Jbuf;
    {
      const int p = tid >> 3, sub = tid & 7;
      const bool valid = p < tl.count;
      const bool ren = tl.term == 1;
      const float deds = xyz[p * 4 + 3];
      const float* gi = gin + p * GIN_PITCH;
      for (int e = sub; e < NPAR; e += 8) {
        float v;
        if (e >= NPOSE) {
          v = ren ? deds * gi[e - NPOSE] : gi[e - NPOSE];
        } else {
          const float g0 = ren ? deds * gi[64] : gi[64];
          const float g1 = ren ? deds * gi[65] : gi[65];
          const float g2 = ren ? deds * gi[66] : gi[66];
          const float x = xyz[p * 4 + 0], y = xyz[p * 4 + 1], z = xyz[p * 4 + 2];
          // g . [I | -[x]x | x]  (get_points_to_pose_jacobian_sim3, loss_utils.py:176-195)
          switch (e) {
            case 0: v = g0; break;
            case 1: v = g1; break;
            case 2: v = g2; break;
            case 3: v = g1 * (-z) + g2 * y; break;
            case 4: v = g0 * z + g2 * (-x); break;
            case 5: v = g0 * (-y) + g1 * x; break;
            default: v = (g0 * x + g1 * y) + g2 * z; break;
          }
        }
        J[p * JPITCH + e] = valid ? v : 0.f;
      }
      if (tid < TILE) {
        // Huber-weighted residual (loss_utils.py:246-275); sdf residual = decoder output
        const float res = ren ? rs[tid] : ys[tid];
        const float b = ren ? P.b1 : P.b2;
        const float x = fabsf(res);
        const float hn = (x <= b) ? x * x : (2.0f * b) * x - b * b;
        const float den = (x == 0.f) ? 1.f : x;
        const float wgt = sqrtf(hn) / den;
        const float rt = (tid < tl.count) ? (P.raw_residual ? res : wgt * res) : 0.f;
        rs[tid] = rt;
        J[tid * JPITCH + NPAR] = rt;           // [J | r~]: column 71 (the pitch pad)
        if (res_out && !ren && tid < tl.count) res_out[d.pts_off + tl.start + tid] = res;
      }
    }
    __syncthreads();
    // ---- per-tile partials: upper-tri J^T J, J^T r~, sum r~^2 = the upper triangle of
    // [J | r~]^T [J | r~] (64 x 72 in LDS): J^T J at (a, b < 71), J^T r~ at (a, 71), sum r~^2 at
    // (71, 71); 15 upper-triangle 16x16 blocks of the padded 80 x 80 product on fp32 MFMA.
    // v_mfma_f32_16x16x4_f32 is an exact fp32 fma chain over its 4 k values in lane-group
    // order (MI355X_MICROARCH.md §Matrix cores), and chunk c holds points 4c..4c+3, so every sum
    // runs over p = 0..63 in order from 0: bitwise the per-element fmaf loop it replaces.
    // (Rows/columns 72..79 read past the pad into the next row: garbage that reaches only
    // outputs at a or b >= 72, which are never stored.)
    {
      const int slot = d.slot_sdf + (tl.term == 0 ? 0 : st[tl.obj].n_sdf_tiles) + tl.start / TILE;
      float* out = slots + (size_t)slot * SLOT_FLOATS;
      const int wv = tid >> 6, lane = tid & 63, i = lane & 15, g = lane >> 4;
      for (int blk = wv; blk < 15; blk += 8) {
        int rb = 0, rem = blk;
        while (rem >= 5 - rb) { rem -= 5 - rb; ++rb; }
        const int cb = rb + rem;
        const float* Ja = J + g * JPITCH + 16 * rb + i;
        const float* Jb = J + g * JPITCH + 16 * cb + i;
        floatx4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int c = 0; c < TILE / 4; ++c)
          acc = __builtin_amdgcn_mfma_f32_16x16x4f32(Ja[4 * c * JPITCH], Jb[4 * c * JPITCH], acc, 0, 0, 0);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int a = 16 * rb + 4 * g + r, b = 16 * cb + i;      // D row 4g + r, column i
          if (a <= b && b <= NPAR) {
            const int e = (b < NPAR) ? a * NPAR - a * (a - 1) / 2 + (b - a) : (a < NPAR ? NTRI + a : NTRI + NPAR);
            out[e] = accr(acc, r);
          }
        }
      }
    }
    __syncthreads();
}

struct JacShared {
  float H[H_FLOATS];           // activations / gradients, later the tile's J [64][72]
  float xyz[TILE * 4];         // object-frame point (x,y,z) + de_ds (render term)
  float red[NWAVE * TILE];     // lin8 partials
  float y[TILE];               // sdf
  float r[TILE];               // raw residual (render) ; later r~ (Huber-weighted)
  float gin[TILE * GIN_PITCH]; // d sdf / d [code(64), xyz(3)]
};


#ifndef DSR_JAC_VARIANT
#define DSR_JAC_VARIANT 6
#endif
template <int V>
__device__ __forceinline__ void jac_gemm(const float4* A, int T, const float* Hs, floatx4 (&acc)[4][4],
                                         int lane) {
  if constexpr ((V & 2) != 0) gemm_tile_pf<4, (V & 4) != 0>(A, T, Hs, acc, lane);
  else gemm_tile<4>(A, T, Hs, acc, lane);
}

__global__ __launch_bounds__(512) void k_mlp_jac(DevDecoder D, const Tile* __restrict__ tiles,
                                                 const int* __restrict__ n_tiles,
                                                 const ObjDesc* __restrict__ desc,
                                                 const ObjState* __restrict__ st,
                                                 const float* __restrict__ pts_all,
                                                 const float4* __restrict__ kpts,
                                                 const float* __restrict__ kres,
                                                 const float* __restrict__ bias0f,
                                                 const float* __restrict__ bias4f, GNParams P,
                                                 float* __restrict__ slots,
                                                 const float4* __restrict__ raw_pts,
                                                 float* __restrict__ raw_out,
                                                 float* __restrict__ res_out, MaskArgs, float*) {
  __shared__ JacShared sm;
  constexpr int JV = DSR_JAC_VARIANT;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nt = *n_tiles;
  for (int ti = blockIdx.x; ti < nt; ti += gridDim.x) {
    const Tile tl = tiles[ti];
    const ObjDesc d = desc[tl.obj];
    // ---- load points
    if (tid < TILE) {
      float x = 0.f, y = 0.f, z = 0.f, aux = 0.f, rr = 0.f;
      if (tid < tl.count) {
        if (tl.term == 0) {                          // surface points -> object frame (loss.py:31-32)
          const float* p = pts_all + (size_t)(d.pts_off + tl.start + tid) * 3;
          const float3 xo = xform(st[tl.obj].T, p[0], p[1], p[2]);
          x = xo.x; y = xo.y; z = xo.z;
        } else if (tl.term == 1) {
          const float4 v = kpts[d.cand_off + tl.start + tid];
          x = v.x; y = v.y; z = v.z; aux = v.w;
          rr = kres[d.cand_off + tl.start + tid];
        } else {
          const float4 v = raw_pts[tl.start + tid];
          x = v.x; y = v.y; z = v.z;
        }
      }
      sm.xyz[tid * 4 + 0] = x; sm.xyz[tid * 4 + 1] = y;
      sm.xyz[tid * 4 + 2] = z; sm.xyz[tid * 4 + 3] = aux;
      sm.r[tid] = rr;
    }
    __syncthreads();
    // ---- forward, masks kept in registers
    uint64_t mk[8];
    layer0_fwd(D, bias0f + tl.obj * HID, sm.xyz, sm.H, w, lane, mk[0]);
    __syncthreads();
    floatx4 acc[4][4];
#pragma unroll
    for (int l = 1; l <= 6; ++l) {
      const int T = D.Kf[l] / 16;
      jac_gemm<JV>(D.Wf[l] + (size_t)(4 * w) * T * 64, T, sm.H, acc, lane);
      __syncthreads();
      epi_fwd(acc, (l == 4) ? bias4f + tl.obj * HID : D.bias[l], sm.H, sm.xyz, w, lane, mk[l], l == 3, D.l3);
      __syncthreads();
    }
    {
      const int T = D.Kf[7] / 16;
      jac_gemm<JV>(D.Wf[7] + (size_t)(4 * w) * T * 64, T, sm.H, acc, lane);
      epi_l7(acc, D, sm.red, w, lane, mk[7]);
    }
    __syncthreads();
    if (tid < TILE) {
      float s = sm.red[tid];
      for (int k = 1; k < NWAVE; ++k) s += sm.red[k * TILE + tid];
      sm.y[tid] = tanhf(s + D.b8);
    }
    __syncthreads();
    // ---- g7 = (1 - y^2) W8 (.) relu'(a7)  (tanh backward, lin8 backward)
    {
      const int g = lane >> 4, c = lane & 15;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int n0 = 64 * w + 16 * q + 4 * g;
        const float4 w8 = *reinterpret_cast<const float4*>(D.W8 + n0);
#pragma unroll
        for (int cb = 0; cb < 4; ++cb) {
          const int p = 16 * cb + c;
          const float yy = sm.y[p];
          const float dt = 1.f - yy * yy;
          float v[4];
#pragma unroll
          for (int r = 0; r < 4; ++r)
            v[r] = ((mk[7] >> ((q * 4 + cb) * 4 + r)) & 1ull) ? dt * fetch4(w8, r) : 0.f;
          *reinterpret_cast<float4*>(sm.H + p * PITCH + n0) = make_float4(v[0], v[1], v[2], v[3]);
        }
      }
    }
    __syncthreads();
    // ---- backward GEMMs: lin7^T .. lin1^T
#pragma unroll
    for (int l = 7; l >= 1; --l) {
      const int T = D.Kb[l] / 16;
      jac_gemm<JV>(D.Wb[l] + (size_t)(4 * w) * T * 64, T, sm.H, acc, lane);
      __syncthreads();
      if (l == 4) epi_bwd_l4(acc, sm.H, sm.gin, w, lane, mk[3], D.l3, D.Kb[3]);
      else epi_bwd(acc, sm.H, w, lane, mk[l - 1]);
      __syncthreads();
    }
    // ---- lin0^T: d sdf / d input (67 rows) = W0^T g0 + skip part (already in gin)
    if (w < 5) {
      floatx4 a1[1][4];
      gemm_tile<1>(D.Wb[0] + (size_t)w * 32 * 64, 32, sm.H, a1, lane);
      const int g = lane >> 4, c = lane & 15;
#pragma unroll
      for (int cb = 0; cb < 4; ++cb) {
        const int p = 16 * cb + c;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int n = 16 * w + 4 * g + r;
          // (a code_len-32 decoder: code slots 32..63 have zero weights and no lin4 part: 0)
          if (n < IN)
            sm.gin[p * GIN_PITCH + n] = accr(a1[0][cb], r) + ((n >= D.code_len && n < CODE) ? 0.f : sm.gin[p * GIN_PITCH + n]);
        }
      }
    }
    __syncthreads();
    jac_tail(tl, d, st, P, slots, raw_out, res_out, sm.y, sm.gin, sm.xyz, sm.r, sm.H, tid);
  }
}

// ------------------------------------------------------------------------------------
// k_mlp_jac16: the Jacobian kernel on split-fp16 MFMA (dsr_mlp16.hpp); same structure as
// k_mlp_jac, every GEMM operand image carried as scaled hi/lo fp16 pieces with a per-tile
// per-layer power-of-two scale (forward activations and backward gradients alike).
// ------------------------------------------------------------------------------------
struct Jac16Shared {
  _Float16 Hh[TILE * PH];      // hi pieces; later the tile's J [64][72] (fp32)
  _Float16 Hl[TILE * PH];
  float xyz[TILE * 4];
  float red[NWAVE * TILE];
  float red2[NWAVE * TILE];    // LayerNorm decoders' second per-point moment (ln_fwd / ln_bwd)
  float y[TILE];
  float r[TILE];
  float gin[TILE * GIN_PITCH];
  float wmax[NWAVE];
};

// The backward GEMMs (W_l^T) keep their lo products off the running sum (gemm16_sel's LS 2,
// dsr_mlp16.hpp), as the forward ones do: the Jacobian's own rounding bias then no longer dominates its error
// (tools/bias_probe.py: J bias 3.4e-8 -> 2.3e-8 of |J|, random 8.3e-7 -> 5.8e-7; fp32 numpy
// 5.7e-9 / 7.2e-7) — the sum b = sum_p J_p r_p cancels to ~1e-5 of its terms on a converging
// object, so that bias, not the random error, is what its pose rows see.
#if defined(DSR_EXP_NOLS)
constexpr int BWD_LS = 0;
#elif defined(DSR_EXP_BLS1)
constexpr int BWD_LS = 1;
#else
constexpr int BWD_LS = 2;
#endif

// NB: A ring depth of the split GEMMs (gemm16_sel; 0 = the two-set gemm16_tile).  Lane-derived
// values are re-derived per layer from an opaque lane id (dsr_mlp_lite.hpp, "Register
// discipline"); row-selecting conditions are wave-uniform branches + per-lane selects.
#ifdef DSR_EXP_STAMP   // diagnostic build (exp_STAMP.so): per-wave cycles by phase, blocks 0-3
#define JSTAMP(cat)                                                         \
  {                                                                         \
    __builtin_amdgcn_sched_barrier(0);                                      \
    const unsigned long long t_ = __builtin_amdgcn_s_memtime();            \
    jstamp[cat] += t_ - jstamp_last;                                        \
    jstamp_last = t_;                                                       \
    __builtin_amdgcn_sched_barrier(0);                                      \
  }
#else
#define JSTAMP(cat)
#endif
// JSTAMP phases: 0 tile inputs / masks, 1 GEMMs, 2 epilogue compute, 3 scale exchange
// (block_scale: its barrier), 4 split writes, 5 post-write barrier, 6 J tail, 7 other
// VAR: the decoder-variant instantiation (use_tanh / xyz_in_all / LayerNorm, DevDecoder); the
// shipped topology's kernel (VAR false) contains none of their code
template <bool PRIO, int NB, bool VAR = false>
__global__ __launch_bounds__(512) void k_mlp_jac16(DevDecoder D, const Tile* __restrict__ tiles,
                                                   const int* __restrict__ n_tiles,
                                                   const ObjDesc* __restrict__ desc,
                                                   const ObjState* __restrict__ st,
                                                   const float* __restrict__ pts_all,
                                                   const float4* __restrict__ kpts,
                                                   const float* __restrict__ kres,
                                                   const float* __restrict__ bias0f,
                                                   const float* __restrict__ bias4f, GNParams P,
                                                   float* __restrict__ slots,
                                                   const float4* __restrict__ raw_pts,
                                                   float* __restrict__ raw_out,
                                                   float* __restrict__ res_out, MaskArgs MA,
                                                   float* __restrict__ lnws) {
  __shared__ Jac16Shared sm;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // LayerNorm decoders: this workgroup's x^ / rstd workspace (LN_WS_WG floats; null otherwise)
  float* const lnw = lnws ? lnws + (size_t)blockIdx.x * LN_WS_WG : nullptr;
  const int nt = *n_tiles;
#ifdef DSR_EXP_STAMP
  unsigned long long jstamp[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  unsigned long long jstamp_last = __builtin_amdgcn_s_memtime();
  int jtiles = 0;
#endif
  for (int ti = blockIdx.x; ti < nt; ti += gridDim.x) {
    const Tile tl = tiles[ti];
    const ObjDesc d = desc[tl.obj];
#ifdef DSR_EXP_STAMP
    ++jtiles;
#endif
    float zpre = 0.f;   // the code's NaN probe for the tail, loaded now (wave 0)
    {
      const int tid = opaque(threadIdx.x);
      if (tid < TILE) {
        float x = 0.f, y = 0.f, z = 0.f, aux = 0.f, rr = 0.f;
        zpre = bias0f[tl.obj * HID];
        if (tid < tl.count) {
          if (tl.term == 0) {
            const float* p = pts_all + (size_t)(d.pts_off + tl.start + tid) * 3;
            const float3 xo = xform(st[tl.obj].T, p[0], p[1], p[2]);
            x = xo.x; y = xo.y; z = xo.z;
          } else if (tl.term == 1) {
            const float4 v = kpts[d.cand_off + tl.start + tid];
            x = v.x; y = v.y; z = v.z; aux = v.w;
            rr = kres[d.cand_off + tl.start + tid];
          } else {
            const float4 v = raw_pts[tl.start + tid];
            x = v.x; y = v.y; z = v.z;
          }
        }
        *reinterpret_cast<float4*>(sm.xyz + tid * 4) = make_float4(x, y, z, aux);
        sm.r[tid] = rr;
      }
    }
    __syncthreads();
    uint64_t mk[8];
    float v[4][4][4];
    floatx4 acc[4][4];
    int sa;          // backward gradients: one scale per tile and layer
    Scales2 fs;      // forward activations: per-group scales (block_scale2), as the exact pass
    // render points whose ReLU masks and sdf the exact re-decode kept (MaskArgs): only the
    // backward chain runs; otherwise the forward recomputes them (loss.py:157)
    // (sdf tiles: the exact pass ran their forward too, MaskArgs.pts)
    bool fast = false;
    if (MA.kslot != nullptr && tl.term == 1) {
      const int tid = opaque(threadIdx.x);
      int bad = 0;
      if (tid < tl.count) bad = MA.kslot[d.cand_off + tl.start + tid] < 0;
      fast = !__syncthreads_or(bad);
    } else if (MA.pts != nullptr && tl.term == 0) {
      fast = true;
    }
    // absolute mask slot of the tile's point p
    auto mslot = [&](int p) {
      return tl.term == 1 ? d.cand_off + MA.kslot[d.cand_off + tl.start + p] : MA.surf_base + d.pts_off + tl.start + p;
    };
    if (fast) {
      const int lane = opaque(threadIdx.x & 63), g = lane >> 4, c = lane & 15;
#pragma unroll
      for (int l = 0; l < 8; ++l) mk[l] = 0;
#pragma unroll
      for (int cb = 0; cb < 4; ++cb) {
        const int p = 16 * cb + c;
        if (p < tl.count) {   // layers 0..7 of this lane's slice: one 16-byte load (mask_store)
          const uint4 m4 = *reinterpret_cast<const uint4*>(MA.msk + (size_t)mslot(p) * 256 + (w * 4 + g) * 8);
          const unsigned dw[4] = {m4.x, m4.y, m4.z, m4.w};
#pragma unroll
          for (int l = 0; l < 8; ++l) {
            const unsigned u = (dw[l >> 1] >> (16 * (l & 1))) & 0xFFFFu;
#pragma unroll
            for (int q = 0; q < 4; ++q) mk[l] |= (uint64_t)((u >> (4 * q)) & 0xFu) << (16 * q + 4 * cb);
          }
        }
      }
      const int tid = opaque(threadIdx.x);
      if (tid < TILE) sm.y[tid] = (tid < tl.count) ? MA.yv[mslot(tid)] : 0.f;
      __syncthreads();
      JSTAMP(0)
    } else {
      JSTAMP(0)
      // ---- lin0 (VALU, fp32) + masks
      {
        const int lane = opaque(threadIdx.x & 63), g = lane >> 4, c = lane & 15;
        const float* bias0 = bias0f + tl.obj * HID;
        float m = 0.f;
        mk[0] = 0;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int n0 = 64 * w + 16 * q + 4 * g;
          const float4 bb = *reinterpret_cast<const float4*>(bias0 + n0);
          float wx[12];
#pragma unroll
          for (int i = 0; i < 12; ++i) wx[i] = D.W0x[n0 * 3 + i];
#pragma unroll
          for (int cb = 0; cb < 4; ++cb) {
            const float4 p = *reinterpret_cast<const float4*>(sm.xyz + (16 * cb + c) * 4);
#pragma unroll
            for (int r = 0; r < 4; ++r)
              v[q][cb][r] = fetch4(bb, r) + ((wx[3 * r] * p.x + wx[3 * r + 1] * p.y) + wx[3 * r + 2] * p.z);
          }
        }
        if (VAR && (D.ln_mask & 1)) ln_fwd(v, D.ln_g[0], D.ln_b[0], D.ln_dim[0], sm.red, sm.red2, w, lane, lnw);
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
          for (int cb = 0; cb < 4; ++cb)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const float h = fmaxf(v[q][cb][r], 0.f);   // NaN re-imposed after the backward
              if (h > 0.f) mk[0] |= 1ull << ((q * 4 + cb) * 4 + r);
              v[q][cb][r] = h;
              m = fmaxf(m, h);
            }
        if (VAR && D.xyz_all && w == 7) xyz_rows(v, sm.xyz, lane, m, 3);   // xyz_in_all: lin1's input = h0 | xyz
        JSTAMP(7)
        fs = block_scale2(m, sm.wmax, w, lane);
        JSTAMP(3)
        write_split(v, fs.of(w), sm.Hh, sm.Hl, w, lane);
        JSTAMP(4)
      }
      __syncthreads();
      JSTAMP(5)
      // ---- forward lin1..lin6 (masks kept)
#pragma unroll 1
      for (int l = 1; l <= 6; ++l) {
        const int lane = opaque(threadIdx.x & 63), g = lane >> 4;
        gemm16_sel<PRIO, NB, JFWD_LS>(D.Wh_raw[l], w, D.Kf[l] / 32, sm.Hh, sm.Hl, acc, lane, fs.resc());
        JSTAMP(1)
        const float usc = ldexpf(1.f, -(D.sw[l] + fs.b));
        const float* bias = (l == 4) ? bias4f + tl.obj * HID : D.bias[l];
        float m = 0.f;
        uint64_t bits = 0;
        if (VAR && ((D.ln_mask >> l) & 1)) {   // LayerNorm between lin_l and its ReLU: x^, rstd kept for the backward
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const float4 bb = *reinterpret_cast<const float4*>(bias + 64 * w + 16 * q + 4 * g);
#pragma unroll
            for (int cb = 0; cb < 4; ++cb)
#pragma unroll
              for (int r = 0; r < 4; ++r) v[q][cb][r] = __builtin_fmaf(accr(acc[q][cb], r), usc * rc_sign(q, cb), fetch4(bb, r));
          }
          ln_fwd(v, D.ln_g[l], D.ln_b[l], D.ln_dim[l], sm.red, sm.red2, w, lane, lnw + (size_t)l * LN_WS_LAYER);
#pragma unroll
          for (int q = 0; q < 4; ++q)
#pragma unroll
            for (int cb = 0; cb < 4; ++cb)
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                const float h = fmaxf(v[q][cb][r], 0.f);
                if (h > 0.f) bits |= 1ull << ((q * 4 + cb) * 4 + r);
                v[q][cb][r] = h;
                m = fmaxf(m, h);
              }
        } else {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float4 bb = *reinterpret_cast<const float4*>(bias + 64 * w + 16 * q + 4 * g);
#pragma unroll
          for (int cb = 0; cb < 4; ++cb) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const float h = fmaxf(__builtin_fmaf(accr(acc[q][cb], r), usc * rc_sign(q, cb), fetch4(bb, r)), 0.f);
              if (h > 0.f) bits |= 1ull << ((q * 4 + cb) * 4 + r);
              v[q][cb][r] = h;
              m = fmaxf(m, h);
            }
          }
        }
        }
        mk[l] = bits;
        {   // the next layer's input = h | xyz (lin4's; every layer's under xyz_in_all)
          const int xr = VAR ? xyz_row(D, l) : (l == 3 ? D.l3 : -1);
          if (xr >= 0 && w == (xr >> 6)) xyz_rows(v, sm.xyz, lane, m, (xr >> 4) & 3);
        }
        JSTAMP(2)
        fs = block_scale2(m, sm.wmax, w, lane);
        JSTAMP(3)
        write_split(v, fs.of(w), sm.Hh, sm.Hl, w, lane);
        JSTAMP(4)
        __syncthreads();
        JSTAMP(5)
      }
      // ---- lin7 + lin8 dot + tanh
      {
        const int lane = opaque(threadIdx.x & 63);
        gemm16_sel<PRIO, NB, JFWD_LS>(D.Wh_raw[7], w, D.Kf[7] / 32, sm.Hh, sm.Hl, acc, lane, fs.resc());
        JSTAMP(1)
        const int un = D.sw[7] + fs.b;
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
          for (int cb = 0; cb < 4; ++cb)
#pragma unroll
            for (int r = 0; r < 4; ++r) acc[q][cb][r] = ldexpf(acc[q][cb][r], -un) * rc_sign(q, cb);
        const bool ln7 = VAR && ((D.ln_mask >> 7) & 1);
        if (ln7) ln_l7(acc, D, sm.red, sm.red2, w, lane, lnw + (size_t)7 * LN_WS_LAYER);
        epi_l7(acc, D, sm.red, w, lane, mk[7], VAR ? sm.xyz : nullptr, !ln7);
      }
      __syncthreads();
      {
        const int tid = opaque(threadIdx.x);
        if (tid < TILE) {
          float s = sm.red[tid];
          for (int k = 1; k < NWAVE; ++k) s += sm.red[k * TILE + tid];
          float y = tanhf(s + D.b8);
          if (VAR && D.use_tanh) y = tanhf(y);          // use_tanh: lin8 -> tanh -> self.th
          sm.y[tid] = y;
        }
      }
      __syncthreads();
    }
    // xyz_in_all: d sdf / d xyz through the xyz rows of every layer's input (wave 7, block 3,
    // quad 3, r 1..3 — the same lanes that own lin4's xyz rows), summed here, added to gin at lin1
    float xg[4][3] = {{0.f, 0.f, 0.f}, {0.f, 0.f, 0.f}, {0.f, 0.f, 0.f}, {0.f, 0.f, 0.f}};
    const bool xlane = VAR && D.xyz_all && w == 7 && ((threadIdx.x & 63) >> 4) == 3;
    // ---- g7 = (1 - y^2) W8 (.) relu'(a7)   (use_tanh: (1 - y^2)(1 - t^2), t = atanh y = tanh(lin8))
    {
      const int lane = opaque(threadIdx.x & 63), g = lane >> 4, c = lane & 15;
      float m = 0.f;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int n0 = 64 * w + 16 * q + 4 * g;
        const float4 w8 = *reinterpret_cast<const float4*>(D.W8 + n0);
#pragma unroll
        for (int cb = 0; cb < 4; ++cb) {
          const int p = 16 * cb + c;
          const float yy = sm.y[p];
          float dt = 1.f - yy * yy;
          if (VAR && D.use_tanh) {
            const float t = atanhf(yy);
            dt = dt * (1.f - t * t);
          }
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float gv = ((mk[7] >> ((q * 4 + cb) * 4 + r)) & 1ull) ? dt * fetch4(w8, r) : 0.f;
            v[q][cb][r] = gv;
            m = fmaxf(m, fabsf(gv));
            if (q == 3 && r >= 1 && xlane) xg[cb][r - 1] = dt * fetch4(w8, r);   // lin8's xyz columns
          }
        }
      }
      if (VAR && ((D.ln_mask >> 7) & 1))   // through lin7's LayerNorm: dL/da7
        m = ln_bwd(v, D.ln_g[7], D.ln_dim[7], sm.red, sm.red2, w, lane, lnw + (size_t)7 * LN_WS_LAYER);
      JSTAMP(7)
      sa = block_scale(m, sm.wmax, w, lane);     // (no GEMM in flight: the barrier is harmless)
      JSTAMP(3)
      write_split(v, sa, sm.Hh, sm.Hl, w, lane);
      JSTAMP(4)
    }
    __syncthreads();
    JSTAMP(5)
    // ---- backward lin7^T .. lin1^T
#pragma unroll 1
    for (int l = 7; l >= 1; --l) {
      const int lane = opaque(threadIdx.x & 63), g = lane >> 4, c = lane & 15;
      gemm16_sel<PRIO, NB, BWD_LS>(D.Wbh_raw[l], w, D.Kb[l] / 32, sm.Hh, sm.Hl, acc, lane);
      JSTAMP(1)
      const float usc = ldexpf(1.f, -(D.swb[l] + sa));
      float m = 0.f;
      const uint64_t mask = mk[l - 1];
      // element (q, cb, r) = bit (q * 4 + cb) * 4 + r of the mask: compile-time indices
      [&]<int... K>(std::integer_sequence<int, K...>) {
        ([&] {
          constexpr int q = K >> 4, cb = (K >> 2) & 3, r = K & 3;
          const float gv = keep_if<K>(accr(acc[q][cb], r) * (usc * rc_sign(q, cb)), mask);   // exact (power of two)
          v[q][cb][r] = gv;
          m = fmaxf(m, fabsf(gv));
        }(), ...);
      }(std::make_integer_sequence<int, 64>{});
      if (xlane && l != 4) {
        // xyz_in_all: layer l's input rows 509..511 are x, y, z — their gradient joins xg, and
        // they carry no ReLU (zeroed, whatever the mask bit)
#pragma unroll
        for (int cb = 0; cb < 4; ++cb)
#pragma unroll
          for (int r = 1; r < 4; ++r) {
            xg[cb][r - 1] += accr(acc[3][cb], r) * (usc * rc_sign(3, cb));
            v[3][cb][r] = 0.f;
          }
      }
      if (l == 1 && xlane) {   // (lin4's xyz slots were written by these lanes at l == 4)
#pragma unroll
        for (int cb = 0; cb < 4; ++cb)
#pragma unroll
          for (int k = 0; k < 3; ++k) sm.gin[(16 * cb + c) * GIN_PITCH + CODE + k] += xg[cb][k];
      }
      if (l == 4 && w >= (D.l3 >> 6)) {
        // d/d[code, xyz] via the latent skip: lin3^T's input rows n >= l3 (445 at code_len 64:
        // wave 7 all, wave 6 rows 445..447) are lin4's code and xyz columns.  Their gradient
        // goes to gin (gin_slot), and they carry no ReLU (mask bit 0 for them: zeroed)
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
          for (int cb = 0; cb < 4; ++cb) {
            const int p = 16 * cb + c;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int n = 64 * w + 16 * q + 4 * g + r;
              if (n >= D.l3) {
                sm.gin[p * GIN_PITCH + gin_slot(n, D.l3)] = accr(acc[q][cb], r) * (usc * rc_sign(q, cb));
                v[q][cb][r] = 0.f;
              }
            }
          }
      }
      if (VAR && ((D.ln_mask >> (l - 1)) & 1))   // through lin_{l-1}'s LayerNorm: dL/da_{l-1}
        m = ln_bwd(v, D.ln_g[l - 1], D.ln_dim[l - 1], sm.red, sm.red2, w, lane, lnw + (size_t)(l - 1) * LN_WS_LAYER);
      JSTAMP(2)
      sa = block_scale(m, sm.wmax, w, lane);
      JSTAMP(3)
      write_split(v, sa, sm.Hh, sm.Hl, w, lane);
      JSTAMP(4)
      __syncthreads();
      JSTAMP(5)
    }
    // ---- lin0^T (80 rows; waves 0..4): d sdf / d input += W0^T g0
    if (w < 5) {
      const int lane = opaque(threadIdx.x & 63), g = lane >> 4, c = lane & 15;
      floatx4 a1[1][4];
      gemm16_tile<PRIO, 1, 0, (BWD_LS != 0)>(reinterpret_cast<const half8*>(D.Wbh_raw[0]) + (size_t)w * 16 * 2 * 64, 16,
                           sm.Hh, sm.Hl, a1, lane);
      const int un = D.swb[0] + sa;
#pragma unroll
      for (int cb = 0; cb < 4; ++cb) {
        const int p = 16 * cb + c;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int n = 16 * w + 4 * g + r;
          if (n < IN)
            sm.gin[p * GIN_PITCH + n] =
                ldexpf(accr(a1[0][cb], r), -un) * rc_sign(w, cb) +
                ((n >= D.code_len && n < CODE) ? 0.f : sm.gin[p * GIN_PITCH + n]);
        }
      }
    }
    // torch.relu propagates NaN; the v_max ReLUs above do not, and a NaN can only come in
    // through the point or the code: re-impose it on the outputs of such points
    const int tid = opaque(threadIdx.x);
    if (tid < TILE) {
      const float4 p = *reinterpret_cast<const float4*>(sm.xyz + tid * 4);
      const float zprobe = zpre;
      if (p.x != p.x || p.y != p.y || p.z != p.z || zprobe != zprobe) {
        sm.y[tid] = __builtin_nanf("");
        for (int e = 0; e < IN; ++e) sm.gin[tid * GIN_PITCH + e] = __builtin_nanf("");
      }
    }
    __syncthreads();
    JSTAMP(7)
    jac_tail(tl, d, st, P, slots, raw_out, res_out, sm.y, sm.gin, sm.xyz, sm.r,
             reinterpret_cast<float*>(sm.Hh), tid);
    JSTAMP(6)
  }
#ifdef DSR_EXP_STAMP
  if (blockIdx.x < 4 && (threadIdx.x == 0 || threadIdx.x == 256))
    printf("jac_stamp %d %d %d %llu %llu %llu %llu %llu %llu %llu %llu\n", (int)blockIdx.x, w, jtiles, jstamp[0],
           jstamp[1], jstamp[2], jstamp[3], jstamp[4], jstamp[5], jstamp[6], jstamp[7]);
#endif
}
#undef JSTAMP

// lane k (a constant after unrolling) of every quad, to the whole quad (DPP quad_perm)
__device__ __forceinline__ float quad_bcast(float v, int k) {
  switch (k) {
    case 0: return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x00, 0xf, 0xf, false));
    case 1: return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x55, 0xf, 0xf, false));
    case 2: return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xaa, 0xf, 0xf, false));
    default: return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xff, 0xf, 0xf, false));
  }
}

// ------------------------------------------------------------------------------------
// k_solve: optimizer.py:131-194 for one object per workgroup
// ------------------------------------------------------------------------------------
constexpr int SOLVE_THREADS = 320;   // 5 waves: substitutions run 4 lanes per column
constexpr int TRACE_V = 2 * NPAR + 3 + 16 + CODE;   // b, dx, loss, sdf, render, T, z
// trace records per (iteration, object), each a whole number of 128 B lines (like counts)
constexpr int TRACE_H_STRIDE = (NPAR * NPAR + 31) / 32 * 32;
constexpr int TRACE_V_STRIDE = (TRACE_V + 31) / 32 * 32;
constexpr int TRACE_I_STRIDE = 32;

// k_reduce_slots: the per-tile normal-equation partials of each object summed in tile order
// (sdf tiles, render tiles: two fp64 sums per element, rounded once), one thread per element
// and SLOT_BLOCKS workgroups per object, 8 tiles' loads in flight per thread — the same
// sums, in the same order, as one workgroup walking the tiles, without that walk's ~90
// dependent memory latencies per object.  red[o][0][e] = sdf sums, red[o][1][e] = render.
// The first workgroup of each object also records the iteration's work counts
// (counts[it][o][NCOUNT], dsr_batch_stats) before k_solve may end the object.
constexpr int SLOT_BLOCKS = (SLOT_FLOATS + 255) / 256;
constexpr int NCOUNT = 6;
// Per-object records written by concurrently running object groups start on their own 128 B
// line: counts[it][o] is one line, red[o] a whole number of lines.
constexpr int COUNT_STRIDE = 32;
constexpr int SRED_STRIDE = (2 * SLOT_FLOATS + 31) / 32 * 32;

__global__ __launch_bounds__(256) void k_reduce_slots(const ObjDesc* __restrict__ desc,
                                                      const ObjState* __restrict__ st,
                                                      const float* __restrict__ slots, float* __restrict__ red,
                                                      int it, int* __restrict__ counts, int stride) {
  const int o = blockIdx.x / SLOT_BLOCKS;
  const ObjState& S = st[o];
  if (blockIdx.x == o * SLOT_BLOCKS && threadIdx.x == 0) {
    int* c = counts + ((size_t)it * stride + o) * COUNT_STRIDE;
    if (S.status != ST_RUNNING) {               // finished / failed objects did no work
      for (int i = 0; i < NCOUNT; ++i) c[i] = 0;
    } else {
      const bool jac = S.n_ren_tiles > 0 || S.k > 0;
      c[0] = S.n_eval;
      c[1] = jac ? desc[o].n_pts + S.k : 0;
      c[2] = S.n_valid;
      c[3] = S.n_refine;
      c[4] = S.n_audit;
      c[5] = jac ? S.k : 0;                     // render points of c[1] (the rest: surface)
    }
  }
  if (S.status != ST_RUNNING || S.lite_viol > 0) return;
  const int e = (blockIdx.x - o * SLOT_BLOCKS) * 256 + threadIdx.x;
  if (e >= SLOT_FLOATS) return;
  const float* s0 = slots + (size_t)desc[o].slot_sdf * SLOT_FLOATS + e;
  auto sum = [&](int n) {
    double x = 0.0;
    int t = 0;
    for (; t + 8 <= n; t += 8, s0 += 8 * SLOT_FLOATS) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = s0[u * SLOT_FLOATS];
#pragma unroll
      for (int u = 0; u < 8; ++u) x += (double)v[u];
    }
    for (; t < n; ++t, s0 += SLOT_FLOATS) x += (double)*s0;
    return (float)x;
  };
  const float a = sum(S.n_sdf_tiles);
  const float b = sum(S.n_ren_tiles);
  red[(size_t)o * SRED_STRIDE + e] = a;
  red[(size_t)o * SRED_STRIDE + SLOT_FLOATS + e] = b;
}

// Rotation prior (compute_rotation_loss_sim3, loss.py:169-192) at the pre-update pose: returns
// res_rot (0 below 1e-7, where the reference zeroes it) and writes its Jacobian J_rot (slots 3
// and 5; the rest zero).  Evaluated in fp64 from the fp32 inverse(T) (the reference's own
// t_cam_obj, same getrf/getrs as optimizer.py:122): res_rot = 1 + R_co[1][1] is a cancellation
// ~1e-5 that k4 = 1e7 multiplies into b[3:6], and the fp32 chain det -> pow(1/3) -> divide puts
// ~1e-7 of noise into R_co[1][1] (1% of res_rot) — in the reference as much as here; fp64
// removes it (tests/test_gpu_parity.py::test_teacher_forced_steps_no_less_accurate_than_the_reference).
__device__ inline float rotation_prior(const float* Tco, float* jrot) {
  double r3[9];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) r3[i * 3 + j] = (double)Tco[i * 4 + j];
  auto det = [](const double* m) {
    return m[0] * (m[4] * m[8] - m[5] * m[7]) - m[1] * (m[3] * m[8] - m[5] * m[6]) +
           m[2] * (m[3] * m[7] - m[4] * m[6]);
  };
  // torch.det(r_co) ** (1/3) (loss.py:177): NaN for a negative determinant (a reflected pose), and
  // the NaN flows into b as it does there (the next iteration then fails like the reference's);
  // cbrt alone would return a finite negative scale
  const double d0 = det(r3);
  const double sc = d0 < 0.0 ? (double)__builtin_nan("") : cbrt(d0);
  for (int i = 0; i < 9; ++i) r3[i] /= sc;
  const double dr = det(r3);
  const double res_rot = 1.0 - (-r3[1 * 3 + 1]);             // 1 - (R_co e_y).n_g
  for (int i = 0; i < NPOSE; ++i) jrot[i] = 0.f;
  if (res_rot < 1e-7) return 0.f;
  // (R_oc n_g) x e_y = (R_oc[2][1], 0, -R_oc[0][1]), R_oc = adj(R_co) / det(R_co)
  jrot[3] = (float)((r3[0 * 3 + 1] * r3[2 * 3 + 0] - r3[0 * 3 + 0] * r3[2 * 3 + 1]) / dr);   // R_oc[2][1]
  jrot[5] = (float)(-(r3[0 * 3 + 2] * r3[2 * 3 + 1] - r3[0 * 3 + 1] * r3[2 * 3 + 2]) / dr);  // -R_oc[0][1]
  return (float)res_rot;
}
#ifdef DSR_EXP_PRIOR_FP32
// Experiment build only: the reference's own fp32 chain (det -> pow(1/3) -> divide -> inverse),
// round 3's code — DESIGN.md §5 (late round 4) used it to rule the fp64 prior out as the cause
// of kitti5's iteration-1 offset.
__device__ inline float rotation_prior_fp32(const float* Tco, float* jrot) {
  float rco[16], rf[9], roc[9];
  for (int i = 0; i < 16; ++i) rco[i] = Tco[i];
  const float sc = powf(det3(rco), 0.33333334f);
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) rf[i * 3 + j] = rco[i * 4 + j] / sc;
  inv_small<3>(rf, roc);
  const float res_rot = 1.f - (-rf[1 * 3 + 1]);
  for (int i = 0; i < NPOSE; ++i) jrot[i] = 0.f;
  if (res_rot < 1e-7f) return 0.f;
  jrot[3] = roc[2 * 3 + 1];
  jrot[5] = -roc[0 * 3 + 1];
  return res_rot;
}
#endif

// trace_* hold [iteration][stride objects]; the pointers are pre-offset to this launch's
// first object (object groups on concurrent streams, dsr_batch_run).
__global__ __launch_bounds__(SOLVE_THREADS) void k_solve(int n_obj, const ObjDesc* __restrict__ desc,
                                                         ObjState* st, float* __restrict__ zbuf,
                                                         GNParams P, const float* __restrict__ red,
                                                         float* __restrict__ trace_H,
                                                         float* __restrict__ trace_v,
                                                         int* __restrict__ trace_i, int stride) {
  const int o = blockIdx.x;
  ObjState& S = st[o];
  if (S.status != ST_RUNNING) return;
  const int tid = threadIdx.x;
  if (S.lite_viol > 0) {
    // An audited sample's exact class differs from the lite pass's (dsr_mlp16.hpp): some
    // unaudited sample may be misclassified too, so this iteration's terms are not trusted.
    // Discard it — no update, no trace, no failure exit — and redo it with every sample
    // decoded exactly (k_iter_begin); dsr_batch_run enqueues one spare iteration for this.
    if (tid == 0) {
      S.lite_viol_total += S.lite_viol;
      S.lite_redo = 1;
    }
    return;
  }
  const ObjDesc d = desc[o];
  __shared__ float Ss[SLOT_FLOATS];
  __shared__ float Sr[SLOT_FLOATS];
  __shared__ float A[NPAR][NPAR + 1];
  __shared__ float X[NPAR][NPAR + 1];
  __shared__ float bv[NPAR], dx[NPAR], z[CODE];
  __shared__ float jrot[NPOSE];
  __shared__ float scal[4];
  __shared__ int piv[NPAR];
  __shared__ float pivv[NPAR];
  __shared__ int flag;
  constexpr int LP = NPAR + 3;                  // fp64 pitch 74: 16-byte aligned rows (the panel reads)
  __shared__ __attribute__((aligned(16))) double Lc[NPAR + 1][LP];   // Cholesky factor, b as row NPAR
  __shared__ double rdg[NPAR];                  // 1 / L[c][c]
  __shared__ int chol_bad;
#ifdef DSR_SOLVE_PROFILE
  const long long tp0 = wall_clock64();
#endif
  {   // the tile partials' sums (k_reduce_slots): all of a thread's loads issued before its stores
    constexpr int NL = (SLOT_FLOATS + SOLVE_THREADS - 1) / SOLVE_THREADS;
    const float* r = red + (size_t)o * SRED_STRIDE;
    float vs[NL], vr[NL];
#pragma unroll
    for (int q = 0; q < NL; ++q) {
      const int e = min(tid + q * SOLVE_THREADS, SLOT_FLOATS - 1);
      vs[q] = r[e];
      vr[q] = r[SLOT_FLOATS + e];
    }
#pragma unroll
    for (int q = 0; q < NL; ++q) {
      const int e = tid + q * SOLVE_THREADS;
      if (e < SLOT_FLOATS) {
        Ss[e] = vs[q];
        Sr[e] = vr[q];
      }
    }
  }
  if (tid < CODE) z[tid] = zbuf[o * CODE + tid];
  // rotation prior, loss.py:169-192, at the current (pre-update) pose (rotation_prior), by a
  // lane of wave 1 while the loads land (its result is only read when no failure exit is taken)
  if (tid == 64) {
#ifdef DSR_EXP_PRIOR_FP32
    scal[1] = rotation_prior_fp32(S.Tco, jrot);
#else
    scal[1] = rotation_prior(S.Tco, jrot);
#endif
  }
  __syncthreads();
  const int it = S.iters_done;
  if (tid == 0) {
    const float N = (float)d.n_pts, K = (float)S.k;
    const float sdf_loss = Ss[SLOT_FLOATS - 1] / N;
    const float ren_loss = Sr[SLOT_FLOATS - 1] / K;     // K == 0 -> NaN, like mean(empty)
    S.sdf_loss = sdf_loss;
    S.render_loss = ren_loss;
    int f = 0;
    if (sdf_loss != sdf_loss) f = DSR_FAIL_SDF_NAN;                 // optimizer.py:137
    else if (ren_loss != ren_loss) f = DSR_FAIL_RENDER_NAN;         // :151
    flag = f;
    if (f) {
      S.status = ST_FAIL;
      S.fail_reason = f;
    } else {
      scal[0] = P.k1 * ren_loss + P.k2 * sdf_loss;                 // :157
      scal[2] = N;
      scal[3] = K;
    }
  }
  __syncthreads();
  if (flag) return;
  // ---- H, b (optimizer.py:161-186)
  {
    const float N = scal[2], K = scal[3];
    const float k1 = P.k1, k2 = P.k2, k3 = P.k3, k4 = P.k4;
    for (int e = tid; e < NPAR * NPAR; e += SOLVE_THREADS) {
      const int a = e / NPAR, b = e - (e / NPAR) * NPAR;
      const int lo = min(a, b), hi = max(a, b);
      const int idx = lo * NPAR - lo * (lo - 1) / 2 + (hi - lo);
      float h = (k1 * Sr[idx]) / K + (k2 * Ss[idx]) / N;
      if (a >= NPOSE && a == b) h = h + k3;
      if (a < NPOSE && b < NPOSE) {
        h = h + k4 * (jrot[a] * jrot[b]);
        if (a == b) h = h + 1.f;
        if (a == NPOSE - 1 && b == NPOSE - 1) h = h + P.s_damp;
      }
      A[a][b] = h;
      if (b <= a) Lc[a][b] = (double)h;        // the Cholesky's working copy (lower triangle)
    }
    for (int a = tid; a < NPAR; a += SOLVE_THREADS) {
      float v = ((-k1) * Sr[NTRI + a]) / K + ((-k2) * Ss[NTRI + a]) / N;
      if (a >= NPOSE) v = v - k3 * z[a - NPOSE];
      else v = v - k4 * (-(jrot[a] * scal[1]));
      bv[a] = v;
      Lc[NPAR][a] = (double)v;                 // b as row NPAR
    }
    if (tid == 0) chol_bad = 0;
  }
  __syncthreads();
  if (trace_H) {
    for (int e = tid; e < NPAR * NPAR; e += SOLVE_THREADS)
      trace_H[((size_t)it * stride + o) * TRACE_H_STRIDE + e] = A[e / NPAR][e % NPAR];
  }
#ifdef DSR_SOLVE_PROFILE
  const long long tp1 = wall_clock64();
#endif
  // ---- dx = inverse(H) b (optimizer.py:188: torch.inverse(H) then a mat-vec).  H is symmetric
  // positive definite — J^T J / N terms, + I on the pose block, + k3 I on the code block,
  // + s_damp on the scale, + k4 J_rot^T J_rot — so it is solved by a Cholesky factorisation
  // H = L L^T in fp64, with b carried as an extra row of L (row NPAR: the forward substitution
  // L y = b rides along in the factorisation) and one back substitution L^T dx = y: no pivot
  // search, no row swaps, two barriers per 8-column panel (the LU + explicit
  // inverse it replaces took 63 + 21 us per solve, this 13.6 + 3.6).  dx is at least as accurate as the reference's fp32
  // inverse-times-b (tests/test_gpu_parity.py::test_teacher_forced_steps_no_less_accurate_than_
  // the_reference holds it against fp64 truth).  A non-positive or NaN pivot (an H with NaN or
  // inf entries) falls back to the fp32 LU with partial pivoting below, the reference's own
  // getrf / getri arithmetic, so those cases behave exactly as before.
  // a double of lane k as a wave-uniform value (two v_readlane: no LDS round trip)
  auto bcastk = [](double v, int k) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffffll), k), hi = __builtin_amdgcn_readlane((int)(b >> 32), k);
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
  };
  // Blocked right-looking Cholesky with look-ahead, panels of CPW columns.  Wave 0 factors a panel
  // in registers (lane l holds rows c0 + l and c0 + 64 + l; the pivot value and the panel's
  // L[c'][c] reach the other lanes by v_readlane) after applying the previous panel to the
  // panel's own columns itself; meanwhile waves 1-4 apply the previous panel to the rest of the
  // trailing triangle (columns past the new panel, the b row included): one barrier per panel.
  // Every element still takes the panels' updates in panel order, each as the same 8 products
  // subtracted in the same order, so the factors are bitwise those of panel-then-update steps.
  constexpr int CPW = 8;
  static_assert(NPAR % CPW == 7, "last panel width");
  // wave 0: columns [c0, c0 + W) of rows c0..NPAR, first updated by panel [pc, pc + CPW) if pc >= 0
  auto panel = [&](auto WC, int c0, int pc) {
    constexpr int W = decltype(WC)::value;
    const int r0 = c0 + tid, r1 = r0 + 64;
    double a0[W], a1[W];
#pragma unroll
    for (int u = 0; u < W; ++u) {
      a0[u] = (r0 <= NPAR && c0 + u <= r0) ? Lc[r0][c0 + u] : 0.0;
      a1[u] = r1 <= NPAR ? Lc[r1][c0 + u] : 0.0;
    }
    if (pc >= 0) {              // (rows above the diagonal get garbage here: never stored)
      double p0[CPW], p1[CPW];  // this lane's rows of the previous panel
#pragma unroll
      for (int v = 0; v < CPW; ++v) {
        p0[v] = r0 <= NPAR ? Lc[r0][pc + v] : 0.0;
        p1[v] = r1 <= NPAR ? Lc[r1][pc + v] : 0.0;
      }
#pragma unroll
      for (int u = 0; u < W; ++u)
#pragma unroll
        for (int v = 0; v < CPW; ++v) {
          const double lw = Lc[c0 + u][pc + v];
          a0[u] -= p0[v] * lw;
          a1[u] -= p1[v] * lw;
        }
    }
    bool bad = false;
#pragma unroll
    for (int u = 0; u < W; ++u) {
      const double d2 = bcastk(a0[u], u);                   // row c0 + u sits in lane u
      bad = bad || !(d2 > 0.0);
      // 1/sqrt(d2): an fp32 seed (v_rsq_f32, 1 ulp) and two Newton steps in fp64
      double rs = (double)__builtin_amdgcn_rsqf((float)d2);
      const double hd = 0.5 * d2;
      rs = rs * __builtin_fma(-hd * rs, rs, 1.5);
      rs = rs * __builtin_fma(-hd * rs, rs, 1.5);
      a0[u] = (tid == u) ? d2 * rs : a0[u] * rs;
      a1[u] = a1[u] * rs;
      if (tid == 0) rdg[c0 + u] = rs;
#pragma unroll
      for (int w = u + 1; w < W; ++w) {                     // the panel's later columns
        const double lwu = bcastk(a0[u], w);                // L[c0 + w][c0 + u]
        a0[w] -= a0[u] * lwu;
        a1[w] -= a1[u] * lwu;
      }
    }
    if (tid == 0 && bad) chol_bad = 1;
#pragma unroll
    for (int u = 0; u < W; ++u) {
      if (r0 <= NPAR && c0 + u <= r0) Lc[r0][c0 + u] = a0[u];
      if (r1 <= NPAR) Lc[r1][c0 + u] = a1[u];
    }
  };
  if (tid < 64) panel(std::integral_constant<int, CPW>{}, 0, -1);
  __syncthreads();
  for (int c0 = 0; c0 + CPW < NPAR; c0 += CPW) {    // panel [c0, c1) is factored
    const int c1 = c0 + CPW, c2 = min(c1 + CPW, NPAR);
    if (tid < 64) {
      if (c2 - c1 == CPW) panel(std::integral_constant<int, CPW>{}, c1, c0);
      else panel(std::integral_constant<int, NPAR % CPW>{}, c1, c0);
    } else if (c2 < NPAR) {
      // trailing update by panel [c0, c1): A[i][j] -= sum_u L[i][c0+u] L[j][c0+u], c2 <= j <= i,
      // j < NPAR, in 4 x 4 element blocks (block row bi >= block column bj), one per thread of
      // waves 1-4: the 8 panel values of its 4 rows and 4 columns are loaded once (16-byte
      // reads) and reused across the block
      const int nr = NPAR + 1 - c2, nb = (nr + 3) >> 2;
      const int t = tid - 64;
      if (t < nb * (nb + 1) / 2) {
        int bi = (int)((sqrtf(8.f * t + 1.f) - 1.f) * 0.5f);
        while (bi * (bi + 1) / 2 > t) --bi;
        while ((bi + 1) * (bi + 2) / 2 <= t) ++bi;
        const int bj = t - bi * (bi + 1) / 2;
        const int i0 = c2 + 4 * bi, j0 = c2 + 4 * bj;
        double li[4][CPW], lj[4][CPW];
#pragma unroll
        for (int m = 0; m < 4; ++m) {
          const int i = min(i0 + m, NPAR), j = min(j0 + m, NPAR);
#pragma unroll
          for (int u = 0; u < CPW; u += 2) {
            const double2 vi = *reinterpret_cast<const double2*>(&Lc[i][c0 + u]);
            const double2 vj = *reinterpret_cast<const double2*>(&Lc[j][c0 + u]);
            li[m][u] = vi.x; li[m][u + 1] = vi.y;
            lj[m][u] = vj.x; lj[m][u + 1] = vj.y;
          }
        }
        // the block's 16 elements: all loaded, then updated, then stored (no load waits behind a
        // store to a possibly aliasing element); outside the triangle a thread reads / writes its
        // own padding slot of row NPAR (columns NPAR..LP-1 are never read as data)
        double acc[4][4];
        double* const pad = &Lc[NPAR][NPAR + (tid & 1)];
#pragma unroll
        for (int m = 0; m < 4; ++m)
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int i = i0 + m, j = j0 + q;
            acc[m][q] = *((i <= NPAR && j < NPAR && j <= i) ? &Lc[i][j] : pad);
          }
#pragma unroll
        for (int m = 0; m < 4; ++m)
#pragma unroll
          for (int q = 0; q < 4; ++q)
#pragma unroll
            for (int u = 0; u < CPW; ++u) acc[m][q] -= li[m][u] * lj[q][u];
#pragma unroll
        for (int m = 0; m < 4; ++m)
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int i = i0 + m, j = j0 + q;
            *((i <= NPAR && j < NPAR && j <= i) ? &Lc[i][j] : pad) = acc[m][q];
          }
      }
    }
    __syncthreads();
  }
#ifdef DSR_SOLVE_PROFILE
  const long long tp2 = wall_clock64();
#endif
  if (!chol_bad) {
    if (tid < 64) {            // L^T dx = y (row NPAR of L), one dependent step per row, wave 0
      // every L value a lane will use is loaded first (its column of L^T and 1 / L[r][r]), so
      // the dependent chain per row is register-only: x_k = y_k / L[k][k] on lane k, v_readlane,
      // one fma per lane
      const int r0 = tid, r1 = tid + 64;
      constexpr int N1 = NPAR - 64;
      double l0[NPAR], l1[N1];
#pragma unroll
      for (int kk = 0; kk < NPAR; ++kk) l0[kk] = Lc[kk][r0];
#pragma unroll
      for (int kk = 0; kk < N1; ++kk) l1[kk] = Lc[64 + kk][min(r1, NPAR - 1)];
      const double d0 = rdg[r0], d1 = rdg[min(r1, NPAR - 1)];
      double y0 = Lc[NPAR][r0], y1 = r1 < NPAR ? Lc[NPAR][r1] : 0.0;
#pragma unroll
      for (int kk = NPAR - 1; kk >= 0; --kk) {
        const double xk = kk < 64 ? bcastk(y0 * d0, kk) : bcastk(y1 * d1, kk - 64);
        if (r0 == kk) y0 = xk;
        else if (r0 < kk) y0 -= l0[kk] * xk;
        if (kk >= 64) {
          if (r1 == kk) y1 = xk;
          else if (r1 < kk) y1 -= l1[kk - 64] * xk;
        }
      }
      dx[r0] = (float)y0;
      if (r1 < NPAR) dx[r1] = (float)y1;
    }
    __syncthreads();
  } else {
    // ---- LU with partial pivoting (torch.inverse, optimizer.py:188): 2 barriers per pivot.
    // Pivot search of column k: first max |A[r][k]|, r >= k (LAPACK getrf), by wave 0, fused
    // into the previous step's update of column k.  Per step: (X) row swap + column scale,
    // (Y) rank-1 update; the arithmetic is getf2's (multiplier by reciprocal, one fma per
    // element), so the factors are bitwise those of the 4-phase schedule.
    // One 64-bit key per candidate: |v| bits (order-preserving for |v| >= 0) over 0xffff - row
    // (ties: the first row); NaN rows key 0, never chosen (fabsf(NaN) > best is false).  The
    // wave max (DPP reduction) is the first max; its signed value is read back from A, which
    // wave 0 wrote before (LDS keeps a wave's accesses in order).
    auto pivot_search = [&](int k, int r0, float v0, int r1, float v1) {   // wave 0, lanes' candidates
      auto key = [](float v, int r) -> unsigned long long {
        const float a = fabsf(v);
        return (r < NPAR && a >= 0.f) ? ((unsigned long long)__float_as_uint(a) << 32) | (unsigned)(0xffff - r) : 0ull;
      };
      const unsigned long long k0 = key(v0, r0), k1 = key(v1, r1);
      const unsigned long long km = __ockl_wfred_max_u64(k0 > k1 ? k0 : k1);
      if (tid == 0) {
        const int bi = km ? 0xffff - (int)(km & 0xffffffffull) : NPAR;
        piv[k] = bi;
        pivv[k] = bi < NPAR ? A[bi][k] : 0.f;
      }
    };
    if (tid < 64) pivot_search(0, tid, A[tid][0], tid + 64, tid + 64 < NPAR ? A[tid + 64][0] : 0.f);
    __syncthreads();
    for (int k = 0; k < NPAR; ++k) {
      const int p = piv[k];
      {   // (X) swap rows k, p (every column but k); column k: pivot to the diagonal, scale below
        const float pv = pivv[k];                            // = A[p][k] (written below)
        const float rc = 1.0f / pv;
        for (int c = tid; c < NPAR; c += SOLVE_THREADS)
          if (c != k && p != k) { const float t = A[k][c]; A[k][c] = A[p][c]; A[p][c] = t; }
        for (int r = k + 1 + tid; r < NPAR; r += SOLVE_THREADS) {
          const float x = (r == p) ? A[k][k] : A[r][k];      // post-swap row r's column-k value
          A[r][k] = x * rc;
          if (r == p) A[k][k] = pv;
        }
      }
      __syncthreads();
      {   // (Y) trailing update; wave 0 owns column k+1 and searches its pivot
        const int m = NPAR - k - 1;
        if (tid < 64) {
          if (k + 1 < NPAR) {
            const int c = k + 1;
            const int r0 = k + 1 + tid, r1 = r0 + 64;
            float v0 = 0.f, v1 = 0.f;
            if (r0 < NPAR) { v0 = __builtin_fmaf(-A[r0][k], A[k][c], A[r0][c]); A[r0][c] = v0; }
            if (r1 < NPAR) { v1 = __builtin_fmaf(-A[r1][k], A[k][c], A[r1][c]); A[r1][c] = v1; }
            pivot_search(k + 1, r0, v0, r1, v1);
          }
        } else if (m > 1) {         // rows k+1.., columns k+2..: a fixed 16 x 16 thread grid
          static_assert(SOLVE_THREADS - 64 == 256, "trailing-update grid");
          const int rr = (tid - 64) >> 4, cc = (tid - 64) & 15;
          for (int r = k + 1 + rr; r < NPAR; r += 16) {
            const float ark = A[r][k];
            for (int c = k + 2 + cc; c < NPAR; c += 16) A[r][c] = __builtin_fmaf(-ark, A[k][c], A[r][c]);
          }
        }
      }
      __syncthreads();
    }
    // inverse(H) = U^-1 L^-1 P I in LDS: the row permutation of the identity, then the
    // forward / back substitutions of getrs, one column per thread (each element
    // accumulates in the column-solve order)
    for (int e = tid; e < NPAR * NPAR; e += SOLVE_THREADS) X[e / NPAR][e % NPAR] = 0.f;
    __syncthreads();
    if (tid < 64) {
      // P applied to the row indices of I: the pivots' swaps in order on a permutation held
      // across wave 0 (lane i: perm[i] and perm[64 + i]) with lane reads / selects — a private
      // array indexed by the run-time pivot would live in scratch memory, one dependent
      // round trip per swap
      static_assert(NPAR <= 128, "permutation held in two registers per lane");
      const int lane = tid;
      int pa = lane, pb = 64 + lane;
      const int qa = piv[lane], qb = (64 + lane < NPAR) ? piv[64 + lane] : 0;
      for (int k = 0; k < NPAR; ++k) {
        const int p = (k < 64) ? __builtin_amdgcn_readlane(qa, k) : __builtin_amdgcn_readlane(qb, k - 64);
        if (p != k) {
          const int vk = (k < 64) ? __builtin_amdgcn_readlane(pa, k) : __builtin_amdgcn_readlane(pb, k - 64);
          const int vp = (p < 64) ? __builtin_amdgcn_readlane(pa, p) : __builtin_amdgcn_readlane(pb, p - 64);
          if (k < 64) pa = (lane == k) ? vp : pa; else pb = (lane == k - 64) ? vp : pb;
          if (p < 64) pa = (lane == p) ? vk : pa; else pb = (lane == p - 64) ? vk : pb;
        }
      }
      X[lane][pa] = 1.f;
      if (64 + lane < NPAR) X[64 + lane][pb] = 1.f;
    }
    __syncthreads();
    // Column c is solved by the 4 lanes 4c..4c+3 of one wave, lane `sub` holding rows
    // i = sub + 4m (m < 18) in registers; a pivot row's value reaches the quad by a DPP
    // broadcast, A is read as LDS broadcasts.  No barriers; each element is updated by one
    // lane in the column-solve order (bitwise the getrs substitutions).
    if (tid < 4 * NPAR) {
      const int c = tid >> 2, sub = tid & 3;
      constexpr int NM = (NPAR + 3) / 4;
      float x[NM];
  #pragma unroll
      for (int m = 0; m < NM; ++m) x[m] = (sub + 4 * m < NPAR) ? X[sub + 4 * m][c] : 0.f;
  #pragma unroll
      for (int l = 0; l < NPAR - 1; ++l) {   // L (unit diagonal): X[i] -= A[i][l] X[l], i > l
        const float xl = quad_bcast(x[l >> 2], l & 3);
  #pragma unroll
        for (int m = l / 4; m < NM; ++m) {
          const int i = sub + 4 * m;
          if (i > l && i < NPAR) x[m] = __builtin_fmaf(-A[i][l], xl, x[m]);
        }
      }
  #pragma unroll
      for (int i = NPAR - 1; i >= 0; --i) {  // U: X[i] /= A[i][i], then X[r] -= A[r][i] X[i], r < i
        const float xi = quad_bcast(x[i >> 2], i & 3) / A[i][i];
        if (sub == (i & 3)) x[i >> 2] = xi;
  #pragma unroll
        for (int m = 0; 4 * m < i; ++m) {
          const int r = sub + 4 * m;
          if (r < i) x[m] = __builtin_fmaf(-A[r][i], xi, x[m]);
        }
      }
  #pragma unroll
      for (int m = 0; m < NM; ++m)
        if (sub + 4 * m < NPAR) X[sub + 4 * m][c] = x[m];
    }
    __syncthreads();
    if (tid < NPAR) {                     // dx = inverse(H) b
      float s = 0.f;
      for (int l = 0; l < NPAR; ++l) s = __builtin_fmaf(X[tid][l], bv[l], s);
      dx[tid] = s;
    }
    __syncthreads();
  }
#ifdef DSR_SOLVE_PROFILE                 // (tools: per-phase wall clock of block 0, 100 MHz ticks)
  const long long tp3 = wall_clock64();
  if (tid == 0 && o == 0) printf("solve_prof %lld %lld %lld\n", tp1 - tp0, tp2 - tp1, tp3 - tp2);
#endif
  if (tid < CODE) zbuf[o * CODE + tid] = z[tid] + P.lr * dx[NPOSE + tid];   // :194
  if (tid == 0) {
    float xi[NPOSE], dT[16], Tn[16], Tprev[16];
    for (int i = 0; i < 16; ++i) Tprev[i] = S.T[i];
    for (int i = 0; i < NPOSE; ++i) xi[i] = P.lr * dx[i];
    exp_sim3_dev(xi, dT);                                         // :190
    mm4(dT, S.T, Tn);                                             // :192
    for (int i = 0; i < 16; ++i) S.T[i] = Tn[i];
    S.loss = scal[0];
    S.iters_done = it + 1;
    if (it + 1 >= P.iters) S.status = ST_DONE;
    if (trace_v) {
      float* tv = trace_v + ((size_t)it * stride + o) * TRACE_V_STRIDE;
      for (int i = 0; i < NPAR; ++i) { tv[i] = bv[i]; tv[NPAR + i] = dx[i]; }
      tv[2 * NPAR + 0] = scal[0];
      tv[2 * NPAR + 1] = S.sdf_loss;
      tv[2 * NPAR + 2] = S.render_loss;
      for (int i = 0; i < 16; ++i) tv[2 * NPAR + 3 + i] = Tprev[i];
      for (int i = 0; i < CODE; ++i) tv[2 * NPAR + 19 + i] = z[i];
    }
  }
  if (trace_i && tid == 0) {
    trace_i[((size_t)it * stride + o) * TRACE_I_STRIDE + 0] = S.n_valid;
    trace_i[((size_t)it * stride + o) * TRACE_I_STRIDE + 1] = S.k;
    trace_i[((size_t)it * stride + o) * TRACE_I_STRIDE + 2] = S.n_eval;
    trace_i[((size_t)it * stride + o) * TRACE_I_STRIDE + 3] = S.n_refine;
  }
}

// ------------------------------------------------------------------------------------
// k_solve_pose: one iteration of Optimizer.estimate_pose_cam_obj (optimizer.py:62-74):
// H = J^T J / N + 1e-2 I (6x6, se3 part of the Sim(3) J), b = -J^T r / N (raw residual),
// dx = inverse(H) b, T <- exp_se3(dx) T.
// ------------------------------------------------------------------------------------
// One workgroup per object (dsr_pose_only_batch); objects with no points left are skipped.
__global__ void k_solve_pose(const ObjDesc* __restrict__ desc, ObjState* st, const float* __restrict__ slots) {
  const int o = blockIdx.x;
  const ObjDesc d = desc[o];
  if (d.n_pts <= 0) return;
  const int n_tiles = (d.n_pts + TILE - 1) / TILE;
  const float* sl = slots + (size_t)d.slot_sdf * SLOT_FLOATS;
  __shared__ float S[SLOT_FLOATS];
  for (int e = threadIdx.x; e < SLOT_FLOATS; e += blockDim.x) {
    double a = 0.0;
    for (int t = 0; t < n_tiles; ++t) a += (double)sl[(size_t)t * SLOT_FLOATS + e];
    S[e] = (float)a;
  }
  __syncthreads();
  if (threadIdx.x != 0) return;
  const float N = (float)d.n_pts;
  float H[36], Hi[36], b[6], dx[6], dT[16], Tn[16];
  for (int a = 0; a < 6; ++a)
    for (int c = 0; c < 6; ++c) {
      const int lo = min(a, c), hi = max(a, c);
      const int idx = lo * NPAR - lo * (lo - 1) / 2 + (hi - lo);
      H[a * 6 + c] = S[idx] / N + ((a == c) ? 1e-2f : 0.f);
    }
  for (int a = 0; a < 6; ++a) b[a] = (-S[NTRI + a]) / N;
  inv_small<6>(H, Hi);
  for (int a = 0; a < 6; ++a) {
    float s = 0.f;
    for (int c = 0; c < 6; ++c) s = __builtin_fmaf(Hi[a * 6 + c], b[c], s);
    dx[a] = s;
  }
  exp_se3_dev(dx, dT);
  mm4(dT, st[o].T, Tn);
  for (int i = 0; i < 16; ++i) st[o].T[i] = Tn[i];
}

__global__ void k_inv_out(int n_obj, const ObjState* __restrict__ st, float* __restrict__ out) {
  const int o = blockIdx.x * blockDim.x + threadIdx.x;
  if (o < n_obj) inv_small<4>(st[o].T, out + 16 * o);
}

// per-iteration counters for the algorithmic-FLOP bookkeeping:
// decoded samples, Jacobian points (N + K), in-ball samples, exact re-decodes, audits, K
__global__ void k_finalize(int n_obj, const ObjState* __restrict__ st, const float* __restrict__ zbuf,
                           dsr_object_out* __restrict__ out) {
  const int o = blockIdx.x * blockDim.x + threadIdx.x;
  if (o >= n_obj) return;
  const ObjState& S = st[o];
  dsr_object_out r;
  r.is_good = (S.status == ST_DONE) ? 1 : 0;
  r.fail_reason = S.fail_reason;
  r.loss = S.loss;
  r.iters_done = S.iters_done;
  r.n_valid_last = S.n_valid;
  r.k_last = S.k;
  inv_small<4>(S.T, r.t_cam_obj);                                  // optimizer.py:202
  for (int i = 0; i < CODE; ++i) r.code[i] = zbuf[o * CODE + i];
  out[o] = r;
}

}  // namespace dsr

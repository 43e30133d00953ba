// dsr_mlp16_st.hpp — the exact pass (k_mlp_fwd16, MSK variant) with staggered wave groups.
//
// Same arithmetic as k_mlp_fwd16 on the ring GEMM (NB 2) with per-group activation scales
// (Scales2): the same MFMAs in the same k order, the same epilogues, the same split scales —
// so the outputs (sdf, kept masks, lite error, audit verdicts) are bitwise those of the
// barrier kernel.  What changes is the synchronisation, as in the lite pass's staggered
// kernel (dsr_mlp_lite.hpp, k_mlp_fwd_lite_st): waves 0-3 (group A: rows 0..255 = the next
// GEMM's k steps 0..7) and waves 4-7 (group B: rows 256..511 = k steps 8..15) synchronise
// through event counters in LDS instead of two block barriers per layer, so one group's
// epilogue (bias, ReLU, masks, its own scale, split writes) overlaps the other group's MFMAs.
// Events (monotonic; each wave adds 1 per event):
//   cH[g]  group g wrote its rows of the current image (+ its scale in sg[g]), or, after
//          lin7, its lin8 partial sums in `red`
//   cM[g]  a wave of group g published its maximum (wmax) for the group's scale
//   cRlo   a wave passed k step 8 of a GEMM (finished reading rows 0..255)
//   cRhi   a wave finished a GEMM
//   cP     a group-A wave reached k step LAG of a GEMM (B starts a GEMM only then)
//   cT[g]  group g's tile inputs are in place;  cE  a group-B wave finished a tile (tail)
// Group A may overwrite its rows once every wave passed step 8 (cRlo), B once every wave
// finished the GEMM (cRhi); a GEMM reads A's rows after cH[A] and B's after cH[B] (group A
// waits for them at step 7, whose last B-fragment prefetch reaches row 256).  Every wait is
// bounded (st_wait): a block that times out marks itself broken and every object it touched
// has its iteration discarded and redone (lite_viol, k_solve) — results are never silently
// wrong.
#pragma once
#include "dsr_mlp16.hpp"
#include "dsr_mlp_lite.hpp"

namespace dsr {

constexpr int FWD16_ST_LAG = 4;

struct Fwd16StShared {
  _Float16 Hh[TILE * PH];
  _Float16 Hl[TILE * PH];
  float xyz[2][TILE * 4];      // per group
  float red[NWAVE * TILE];
  float wmax[NWAVE];
  int sg[2];                   // each group's split scale of the current image
  int cH[2], cM[2], cRlo, cRhi, cP, cT[2], cE, broken, pad[5];
};
static_assert(sizeof(int) * 18 == sizeof(Fwd16StShared) - offsetof(Fwd16StShared, sg), "counter block");

// gemm16_ring (NB 2) with `hook(t)` at the start of every k step and the group-B rescale
// read from `resc` at step 8 (after hook(8)): bitwise the same MFMA sequence.
template <bool PRIO, int T, class Hook>
__device__ __forceinline__ void gemm16_ring_h(const _Float16* Wl, int w, const _Float16* Hh, const _Float16* Hl,
                                              floatx4 (&acc)[4][4], int lane, const float& resc, Hook hook) {
  constexpr int NB = 2;
  const _Float16* base = Wl + (size_t)(4 * w) * T * 2 * 64 * 8;
  const __amdgpu_buffer_rsrc_t rsrc =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<_Float16*>(base), 0, 4 * T * 2 * 1024, 0x00020000);
  const int voff = lane * 16;
  const int boff = h_boff(lane);
  const _Float16* Bh = Hh + boff;
  const _Float16* Bl = Hl + boff;
  auto lda = [&](int q, int t, int piece) {
    return __builtin_bit_cast(
        half8, __builtin_amdgcn_raw_buffer_load_b128(rsrc, voff, ((q * T + t) * 2 + piece) * 1024, 0));
  };
  half8 ah[NB][4], al[NB][4], bh[2], bl[2];
  hook(0);
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    ah[0][q] = lda(q, 0, 0);
    al[0][q] = lda(q, 0, 1);
  }
  bh[0] = *reinterpret_cast<const half8*>(Bh);
  bl[0] = *reinterpret_cast<const half8*>(Bl);
  auto step = [&](auto J, auto FIRST, int t) {
    constexpr int j = decltype(J)::value;
    if (!decltype(FIRST)::value) hook(t);
    if (t + 1 < T) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        ah[(j + 1) % NB][q] = lda(q, t + 1, 0);
        al[(j + 1) % NB][q] = lda(q, t + 1, 1);
      }
    }
    if (!decltype(FIRST)::value && t == 8 && resc != 1.f) rescale_acc<4>(acc, resc);
    if (PRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int cb = 0; cb < 4; ++cb) {
      const int nk = (cb < 3) ? (cb + 1) * 16 * PH + 32 * t : 32 * (t + 1);
      bh[(cb + 1) & 1] = *reinterpret_cast<const half8*>(Bh + nk);
      bl[(cb + 1) & 1] = *reinterpret_cast<const half8*>(Bl + nk);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        floatx4 x = decltype(FIRST)::value ? floatx4{0.f, 0.f, 0.f, 0.f} : acc[q][cb];
        x = __builtin_amdgcn_mfma_f32_16x16x32_f16(al[j][q], bh[cb & 1], x, 0, 0, 0);
        x = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[j][q], bl[cb & 1], x, 0, 0, 0);
        acc[q][cb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[j][q], bh[cb & 1], x, 0, 0, 0);
      }
    }
    if (PRIO) __builtin_amdgcn_s_setprio(0);
  };
  step(std::integral_constant<int, 0>{}, std::true_type{}, 0);
#pragma unroll 1
  for (int t0 = 1; t0 < T - 1; t0 += 2) {
    step(std::integral_constant<int, 1>{}, std::false_type{}, t0);
    step(std::integral_constant<int, 0>{}, std::false_type{}, t0 + 1);
  }
  step(std::integral_constant<int, 1>{}, std::false_type{}, T - 1);
}

template <bool PRIO, int X>
__global__ __launch_bounds__(512) void k_mlp_fwd16_st(DevDecoder D, const Tile* __restrict__ tiles,
                                                      const int* __restrict__ n_tiles,
                                                      const ObjDesc* __restrict__ desc,
                                                      const float4* __restrict__ cand,
                                                      const float* __restrict__ bias0f,
                                                      const float* __restrict__ bias4f,
                                                      float* __restrict__ dense, unsigned* __restrict__,
                                                      ErtArgs E, MaskArgs MA) {
  static_assert((X & 512) != 0, "staggered exact pass: the kept-mask (MSK) variant");
  __shared__ Fwd16StShared sm;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int grp = w >> 2;
  const int nt = *n_tiles;
  {
    const int tid = opaque(threadIdx.x);
    if (tid < 18) (&sm.sg[0])[tid] = 0;   // sg, counters, broken, pad
  }
  __syncthreads();                         // the only block-wide barrier
  int it = 0;
  for (int ti = blockIdx.x; ti < nt; ti += gridDim.x, ++it) {
    const Tile tl = tiles[ti];
    const ObjDesc d = desc[tl.obj];
    const bool surf = tl.term == 3;
    const int mbase = surf ? MA.surf_base + d.pts_off + tl.start : d.cand_off + tl.start;
    float* xyz = sm.xyz[grp];
    // ---- tile inputs, per group (B's copy is read by its tail until every B wave is done)
    float zpre = 0.f, ylpre = 0.f;     // the tail's global inputs (wave 4)
    {
      if (grp == 1) st_wait(&sm.cE, 4 * it, &sm.broken);
      const int gt = opaque(threadIdx.x) & 255;
      if (gt < TILE) {
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (grp == 1) zpre = bias0f[tl.obj * HID];
        if (gt < tl.count) {
          if (surf) {
            const float* p = MA.pts + (size_t)(d.pts_off + tl.start + gt) * 3;
            const float3 xo = xform(E.st[tl.obj].T, p[0], p[1], p[2]);
            v = make_float4(xo.x, xo.y, xo.z, 0.f);
          } else {
            v = cand[d.cand_off + tl.start + gt];
            if (grp == 1 && E.st) ylpre = dense[d.cand_off + (__float_as_int(v.w) & ~AUDIT_BIT)];
          }
        }
        *reinterpret_cast<float4*>(xyz + gt * 4) = v;
      }
      st_signal(&sm.cT[grp]);
      st_wait(&sm.cT[grp], 4 * (it + 1), &sm.broken);
    }
    MaskQueue mq;
    // group exchange of this layer's maxima -> the group's split scale (event ne, 0-based)
    auto group_scale = [&](float m, int ne, int lane) {
      m = wave_max(m, lane);
      if (lane == 0) sm.wmax[w] = m;
      st_signal(&sm.cM[grp]);
      st_wait(&sm.cM[grp], 4 * (ne + 1), &sm.broken);
      float mm = sm.wmax[4 * grp];
#pragma unroll
      for (int k = 1; k < 4; ++k) mm = fmaxf(mm, sm.wmax[4 * grp + k]);
      return group_scale_exp(mm);
    };
    // write the group's rows of a new image once every reader of the old one is past them
    // (gn: the reading GEMM's number), then publish the rows and the group's scale
    auto publish = [&](const float (&v)[4][4][4], int s, int gn, int lane) {
      st_wait(grp == 0 ? &sm.cRlo : &sm.cRhi, 8 * gn, &sm.broken);
      write_split(v, s, sm.Hh, sm.Hl, w, lane);
      if (w == 4 * grp && lane == 0) sm.sg[grp] = s;
      st_signal(&sm.cH[grp]);
    };
    // ---- lin0 on VALU (fp32), then split
    {
      const int lane = opaque(threadIdx.x & 63), g = lane >> 4, c = lane & 15;
      const float* bias0 = bias0f + tl.obj * HID;
      float v[4][4][4];
      float m = 0.f;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int n0 = 64 * w + 16 * q + 4 * g;
        const float4 bb = *reinterpret_cast<const float4*>(bias0 + n0);
        float wx[12];
#pragma unroll
        for (int i = 0; i < 12; ++i) wx[i] = D.W0x[n0 * 3 + i];
#pragma unroll
        for (int cb = 0; cb < 4; ++cb) {
          const float4 p = *reinterpret_cast<const float4*>(xyz + (16 * cb + c) * 4);
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float a = fetch4(bb, r) + ((wx[3 * r] * p.x + wx[3 * r + 1] * p.y) + wx[3 * r + 2] * p.z);
            v[q][cb][r] = fmaxf(a, 0.f);
            m = fmaxf(m, v[q][cb][r]);
          }
        }
      }
      const int s = group_scale(m, 7 * it, lane);
      publish(v, s, 7 * it, lane);                  // readers: the previous tile's lin7 GEMM
      mask_push(mq, relu_bits(v));
    }
    floatx4 acc[4][4];
    // one GEMM (layer l = 1..7) on the current image; returns the group-B scale sB of its input
    auto gemm = [&](int l, int lane) {
      const int gn = 7 * it + (l - 1);             // GEMMs before this one
      const int hs = 4 * (8 * it + l);             // cH count once the input image is complete
      st_wait(&sm.cH[0], hs, &sm.broken);
      int sA = sm.sg[0], sB = 0;
      float resc = 1.f;
      if (grp == 1) {
        st_wait(&sm.cH[1], hs, &sm.broken);
        st_wait(&sm.cP, 4 * (gn + 1), &sm.broken);
        sB = sm.sg[1];
        resc = ldexpf(1.f, sB - sA);
      }
      auto hook = [&](int t) {
        if (t == 7 && grp == 0) {
          st_wait(&sm.cH[1], hs, &sm.broken);
          sB = sm.sg[1];
          resc = ldexpf(1.f, sB - sA);
        }
        if (t == 8) st_signal(&sm.cRlo);
        if (t == FWD16_ST_LAG && grp == 0) st_signal(&sm.cP);
      };
      if (D.Kf[l] / 32 != 14) gemm16_ring_h<PRIO, 16>(D.Wh_raw[l], w, sm.Hh, sm.Hl, acc, lane, resc, hook);
      else gemm16_ring_h<PRIO, 14>(D.Wh_raw[l], w, sm.Hh, sm.Hl, acc, lane, resc, hook);
      st_signal(&sm.cRhi);
      return sB;
    };
    // ---- lin1..lin6
#pragma unroll 1
    for (int l = 1; l <= 6; ++l) {
      const int lane = opaque(threadIdx.x & 63), g = lane >> 4;
      const int sB = gemm(l, lane);
      const float usc = ldexpf(1.f, -(D.sw[l] + sB));
      const float* bias = (l == 4) ? bias4f + tl.obj * HID : D.bias[l];
      float v[4][4][4];
      float m = 0.f;
      uint64_t bits = 0;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float4 bb = *reinterpret_cast<const float4*>(bias + 64 * w + 16 * q + 4 * g);
#pragma unroll
        for (int cb = 0; cb < 4; ++cb) {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float x = fmaxf(__builtin_fmaf(accr(acc[q][cb], r), usc, fetch4(bb, r)), 0.f);
            if (x > 0.f) bits |= 1ull << ((q * 4 + cb) * 4 + r);
            v[q][cb][r] = x;
            m = fmaxf(m, x);
          }
        }
      }
      if (l == 3 && w == 6) xyz_rows(v, xyz, lane, m);     // lin4 input = h3 | xyz (group B)
      const int s = group_scale(m, 7 * it + l, lane);
      publish(v, s, 7 * it + l, lane);                    // readers: this GEMM (number 7 it + l - 1)
      mask_push(mq, bits);
    }
    // ---- lin7 + the lin8 partial sums
    {
      const int lane = opaque(threadIdx.x & 63);
      const int sB = gemm(7, lane);
      const int un = D.sw[7] + sB;
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int cb = 0; cb < 4; ++cb)
#pragma unroll
          for (int r = 0; r < 4; ++r) acc[q][cb][r] = ldexpf(acc[q][cb][r], -un);
      uint64_t mask;
      epi_l7(acc, D, sm.red, w, lane, mask);
      mask_push(mq, mask);
      mask_store(mq, MA.msk, mbase, tl.count, w, lane);
      st_signal(&sm.cH[grp]);
    }
    // ---- tail (wave 4: the tile's 64 points), then B's tile-done event
    if (grp == 1) {
      if (w == 4) {
        st_wait(&sm.cH[0], 4 * (8 * it + 8), &sm.broken);
        st_wait(&sm.cH[1], 4 * (8 * it + 8), &sm.broken);
        const int lane = opaque(threadIdx.x & 63);
        const int tid = lane;
        const bool broken = __builtin_amdgcn_readfirstlane(sm.broken) != 0;
        float emax = 0.f;
        if (tid < tl.count) {
          float s = sm.red[tid];
          for (int k = 1; k < NWAVE; ++k) s += sm.red[k * TILE + tid];
          float y = tanhf(s + D.b8);
          const float4 p = *reinterpret_cast<const float4*>(xyz + tid * 4);
          if (p.x != p.x || p.y != p.y || p.z != p.z || zpre != zpre) y = __builtin_nanf("");
          if (surf) {
            MA.yv[mbase + tid] = y;
          } else {
            const int tagged = __float_as_int(p.w);
            const int idx = tagged & ~AUDIT_BIT;
            if (E.st) {
              const float e = fabsf(y - ylpre);
              if (e == e) emax = e;
              if (tagged & AUDIT_BIT) {
                const int cl = ylpre <= E.nth ? 0 : (ylpre < -E.nth ? 1 : 2);
                const int ce = y <= E.nth ? 0 : (y < -E.nth ? 1 : 2);
                if (cl != ce) atomicAdd(&E.st[tl.obj].lite_viol, 1);
              }
            }
            dense[d.cand_off + idx] = y;
            MA.yv[d.cand_off + tl.start + tid] = y;
            if (E.dead && y <= E.nth) E.dead[d.ray_off + idx / E.M] = 1;
          }
        }
        if (E.st && !surf) {
          emax = wave_max(emax, lane);
          if (lane == 0 && emax > 0.f) atomicMax(reinterpret_cast<int*>(&E.st[tl.obj].lite_err), __float_as_int(emax));
        }
        // a timed-out wait anywhere in this block: the tile's values are not trusted — the
        // object's iteration is discarded and redone (k_solve, as for an audit violation)
        if (broken && lane == 0 && E.st) atomicAdd(&E.st[tl.obj].lite_viol, 1);
      }
      st_signal(&sm.cE);
    }
  }
}

}  // namespace dsr

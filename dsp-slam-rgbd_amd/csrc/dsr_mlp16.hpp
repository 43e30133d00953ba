// dsr_mlp16.hpp — the decoder forward on split-fp16 MFMA ("3xFP16"), fp32-class accuracy.
//
// Every fp32 GEMM operand x is carried as two IEEE fp16 pieces, x*2^s = hi + lo with
// hi = fp16(x*2^s), lo = fp16(x*2^s - hi) (power-of-two scale s, exact), and
//     A.B = 2^-(sa+sb) (A_hi.B_hi + A_hi.B_lo + A_lo.B_hi)
// on v_mfma_f32_16x16x32_f16 with fp32 accumulation.  Each piece holds 11 significant
// bits, so the pair carries 22; products of fp16 are exact in fp32, the dropped
// A_lo.B_lo term is ~2^-22 relative — the same construction as 3xTF32 (TF32 also has
// an 11-bit significand), i.e. fp32-class results at 3 MFMAs of 16 cycles per
// 16x16x32 block versus 8 f32 MFMAs of 32 cycles: 5.3x the fp32 MFMA rate.
// Scales: weights per layer at load time (max |W| * 2^sw < 2^15), activations per tile
// and layer from the tile's own max (computed in the epilogue, one LDS max-reduction
// that rides on the barrier the epilogue already has) — so no input can overflow fp16
// and small values keep their relative precision.
//
// Layout: LDS holds two images Hh/Hl [64 points][528 halfs] (pitch 528: conflict-free
// ds_read_b128 B-fragment reads).  A fragments are pre-packed per (row block, 32-k step,
// piece): one 1 KiB coalesced wave-load each.  Wave w owns rows 64w..64w+63 as 4x4
// 16x16 accumulators, exactly like the fp32 kernel (dsr_mlp.hpp), so the epilogues and
// the lin8 fusion are shared in structure.
#pragma once
#include <utility>
#include "dsr_dev.hpp"
#include "dsr_mlp.hpp"

namespace dsr {

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef _Float16 half4 __attribute__((ext_vector_type(4)));

constexpr int PH = 528;                      // LDS pitch of the fp16 images (halfs)

// Sign-alternated rows (SPLIT_ROW_SIGNS).  v_mfma_f32_16x16x32_f16 does not round its k-sum
// once: it rounds toward -inf slightly more often than up — a mean of -0.02 .. -0.05 ulp of the
// largest term per instruction where the products dominate (tools/mfma_numerics.py,
// tools/mfma_bias.py).  After a ReLU every activation is >= 0, so "toward -inf" acts as a scale
// (1 - eps) on each layer's live outputs, the layers compound it, and lin8's sum S near the
// surface (~ -b8, 0.63 for the bench decoder) carried it into every sdf: -7.6e-8 on every point,
// 1 ulp of S, against -8e-10 for the fp32-MFMA kernels (tools/bias_probe.py) — and b = sum J r
// (optimizer.py:163-169) adds a common offset up coherently over the N surface points.  So the
// split weights are packed with every odd 16-row block negated (pack_frag16), those rows'
// accumulators hold -(W h), their rounding leans the other way, and the epilogues multiply them
// back by row_sign(q) (exact) — half the rows lean up, half down, and no scale survives.  Zero
// cost: the sign rides on the epilogue's existing unscale multiply.  The lite pass reads its own
// unsigned fp16 copy (Wl_raw); the DSR_LITE_EXPERIMENTS build (whose old lite variants read the
// hi pieces) and DSR_EXP_NOSIGN (A/B) pack without signs.
#if defined(DSR_LITE_EXPERIMENTS) || defined(DSR_EXP_NOSIGN)
constexpr bool SPLIT_ROW_SIGNS = false;
#else
constexpr bool SPLIT_ROW_SIGNS = true;
#endif
// the sign of 16-row block q (rows 64w + 16q .. +15) of a packed split matrix; for lin0^T's
// 80-row pack, whose wave w owns rows 16w .. 16w + 15, pass w
__device__ __forceinline__ constexpr float row_sign(int q) { return (SPLIT_ROW_SIGNS && (q & 1)) ? -1.f : 1.f; }
// Row signs alone leave each point's sdf off by eps * (S_even - S_odd) (the two row halves' shares
// of lin8's sum), -2e-8 on the bench decoder, with lo products chained onto the running sum.
// Chained from zero instead (LS below) the lean is gone (+2e-9, tools/bias_probe.py).  A column
// sign as well (odd 16-point blocks negated: a checkerboard, measured in round 5) cancelled that
// lean over points, but made a point's result depend on its slot in the tile — the lite pass's
// band re-decode, a re-run from a saved state and an 8-rank shard then disagreed with the exact
// pass in the last bits (test_gpu_parity.py's bitwise checks) — so it is not built;
// DSR_EXP_COLSIGN (A/B) restores it.
#ifdef DSR_EXP_COLSIGN
__device__ __forceinline__ constexpr float col_sign(int cb) { return (SPLIT_ROW_SIGNS && (cb & 1)) ? -1.f : 1.f; }
#else
__device__ __forceinline__ constexpr float col_sign(int) { return 1.f; }
#endif
__device__ __forceinline__ constexpr float rc_sign(int q, int cb) { return row_sign(q) * col_sign(cb); }

struct Fwd16Shared {
  _Float16 Hh[TILE * PH];
  _Float16 Hl[TILE * PH];
  float xyz[TILE * 4];
  float red[NWAVE * TILE];
  float red2[NWAVE * TILE];    // LayerNorm decoders' second per-point moment (ln_fwd)
  float wmax[NWAVE];
};

// one 32-k step of the 3-product MFMA block for a 64x64 wave tile
// Hh/Hl images are swizzled: element (point p, k) at p * PH + (k ^ (8 * ((p >> 2) & 1))).
// Unswizzled, the 16-lane groups of write_split's 8-byte stores (16 points of one 4-row
// slice at the 264-dword pitch) hit every bank 4 times; swizzled twice, and the 16-byte B
// reads stay conflict-free (their lane groups mix the two slices).  Readers: the lane's
// B base offset below; writer: write_split.
__device__ __forceinline__ int h_boff(int lane) {
  const int c = lane & 15;
  return c * PH + 8 * ((lane >> 4) ^ ((c >> 2) & 1));
}

// LS: the two lo products of a split GEMM kept off the running sum.  The f16 MFMA rounds each
// 8-deep chunk sum onto its accumulator toward -inf to about an ulp of the ACCUMULATOR
// (tools/mfma_numerics.py): chained onto the large running sum, the two small lo products cost two
// such roundings per k step for ~2^-11 of the product's value.  Measured on one decoder-layer-
// shaped block (tools/split_chain_bias.py): mean error -1.36e-8 of |exact| on the plain chain,
// -1.6e-9 with the lo products from zero, rms 2.4e-7 -> 1.6e-7.  LS 2 (every shipped split GEMM,
// gemm16_ring): the lo products in their own accumulators over the whole k loop, one VALU add per
// output at the end (64 more VGPRs; the kernels fit them: 0 / 36 / 72 B of scratch).  LS 1 (this
// tile path: lin0^T, the NB = 0 A/B kernels): each k step's lo pair chained from zero and added on
// the VALU — 64 adds per k step beside 48 MFMAs, +14% per split launch when every GEMM ran it.
template <bool PRIO, int NQ, int EX = 0, bool LS = false>
__device__ __forceinline__ void mfma3_step(const half8 (&ah)[NQ], const half8 (&al)[NQ], const half8 (&bh)[4],
                                           const half8 (&bl)[4], floatx4 (&acc)[NQ][4]) {
  if (PRIO) __builtin_amdgcn_s_setprio(1);
  if constexpr (LS && (EX & 1) == 0) {
    // per column block: the NQ lo chains side by side, the hi products onto the running sums,
    // then the VALU adds of the lo sums (adding them before the hi product instead is the same
    // arithmetic in another order; measured no faster)
#pragma unroll
    for (int cb = 0; cb < 4; ++cb) {
      floatx4 lo[NQ];
#pragma unroll
      for (int q = 0; q < NQ; ++q)
        lo[q] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al[q], bh[cb], floatx4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
#pragma unroll
      for (int q = 0; q < NQ; ++q) lo[q] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[q], bl[cb], lo[q], 0, 0, 0);
#pragma unroll
      for (int q = 0; q < NQ; ++q)
        acc[q][cb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[q], bh[cb], acc[q][cb], 0, 0, 0) + lo[q];
    }
    if (PRIO) __builtin_amdgcn_s_setprio(0);
    return;
  }
  if constexpr ((EX & 1) == 0) {       // EX bit0: timing experiment, hi.hi product only
#pragma unroll
  for (int q = 0; q < NQ; ++q)
#pragma unroll
    for (int cb = 0; cb < 4; ++cb)
      acc[q][cb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al[q], bh[cb], acc[q][cb], 0, 0, 0);
#pragma unroll
  for (int q = 0; q < NQ; ++q)
#pragma unroll
    for (int cb = 0; cb < 4; ++cb)
      acc[q][cb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[q], bl[cb], acc[q][cb], 0, 0, 0);
  }
#pragma unroll
  for (int q = 0; q < NQ; ++q)
#pragma unroll
    for (int cb = 0; cb < 4; ++cb)
      acc[q][cb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[q], bh[cb], acc[q][cb], 0, 0, 0);
  if (PRIO) __builtin_amdgcn_s_setprio(0);
}

// This wave's slice (row blocks 4w..4w+3) of a packed split-fp16 weight matrix with T k-steps.
__device__ __forceinline__ const half8* wfrag(const _Float16* W, int w, int T) {
  return reinterpret_cast<const half8*>(W) + (size_t)(4 * w) * T * 2 * 64;
}

// First-k-step A fragments of a packed weight matrix (the GEMM's prologue load).
template <int NQ>
__device__ __forceinline__ void load_a0(const half8* __restrict__ A, int T, half8 (&ah)[NQ], half8 (&al)[NQ],
                                        int lane) {
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    ah[q] = A[((q * T) * 2 + 0) * 64 + lane];
    al[q] = A[((q * T) * 2 + 1) * 64 + lane];
  }
}

// acc = A(16*NQ rows of this wave) . H (64 points), K = 32*T.  A: packed [(q*T + t)*2 + piece][lane].
// On entry ah0/al0 hold A's first-k-step fragments; on exit they hold those of the NEXT
// weight matrix An (Tn k-steps), so its L2 latency hides behind this GEMM's last step, the
// epilogue and the barrier instead of stalling the next layer's first MFMA.
template <bool PRIO, int NQ = 4>
__device__ __forceinline__ void gemm16_tile_x(const half8* __restrict__ A, int T, const _Float16* Hh,
                                              const _Float16* Hl, floatx4 (&acc)[NQ][4], int lane,
                                              half8 (&ah0)[NQ], half8 (&al0)[NQ],
                                              const half8* __restrict__ An, int Tn) {
#pragma unroll
  for (int q = 0; q < NQ; ++q)
#pragma unroll
    for (int cb = 0; cb < 4; ++cb) acc[q][cb] = floatx4{0.f, 0.f, 0.f, 0.f};
  const int boff = h_boff(lane);
  const _Float16* Bh = Hh + boff;
  const _Float16* Bl = Hl + boff;
  half8 ah1[NQ], al1[NQ], bh0[4], bl0[4], bh1[4], bl1[4];
#pragma unroll
  for (int cb = 0; cb < 4; ++cb) {
    bh0[cb] = *reinterpret_cast<const half8*>(Bh + cb * 16 * PH);
    bl0[cb] = *reinterpret_cast<const half8*>(Bl + cb * 16 * PH);
  }
  for (int t = 0; t < T; t += 2) {
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      ah1[q] = A[((q * T + t + 1) * 2 + 0) * 64 + lane];
      al1[q] = A[((q * T + t + 1) * 2 + 1) * 64 + lane];
    }
#pragma unroll
    for (int cb = 0; cb < 4; ++cb) {
      bh1[cb] = *reinterpret_cast<const half8*>(Bh + cb * 16 * PH + 32 * (t + 1));
      bl1[cb] = *reinterpret_cast<const half8*>(Bl + cb * 16 * PH + 32 * (t + 1));
    }
    mfma3_step<PRIO, NQ>(ah0, al0, bh0, bl0, acc);
    if (t + 2 < T) {
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        ah0[q] = A[((q * T + t + 2) * 2 + 0) * 64 + lane];
        al0[q] = A[((q * T + t + 2) * 2 + 1) * 64 + lane];
      }
#pragma unroll
      for (int cb = 0; cb < 4; ++cb) {
        bh0[cb] = *reinterpret_cast<const half8*>(Bh + cb * 16 * PH + 32 * (t + 2));
        bl0[cb] = *reinterpret_cast<const half8*>(Bl + cb * 16 * PH + 32 * (t + 2));
      }
    } else {
      load_a0<NQ>(An, Tn, ah0, al0, lane);
    }
    mfma3_step<PRIO, NQ>(ah1, al1, bh1, bl1, acc);
  }
}

// EX: timing experiments only (invalid results): bit0 one MFMA product per block,
// bit1 every k step re-reads the first step's A fragments (no L2 streaming).
// acc *= 2^d (power of two: exact) — the move of the k-steps-0..7 partial sums from group A's
// image scale to group B's at k step 8 (Scales2)
template <int NQ>
__device__ __forceinline__ void rescale_acc(floatx4 (&acc)[NQ][4], float f) {
#pragma unroll
  for (int q = 0; q < NQ; ++q)
#pragma unroll
    for (int cb = 0; cb < 4; ++cb) acc[q][cb] = acc[q][cb] * f;
}

template <bool PRIO, int NQ = 4, int EX = 0, bool LS = false>
__device__ __forceinline__ void gemm16_tile(const half8* __restrict__ A, int T, const _Float16* Hh,
                                            const _Float16* Hl, floatx4 (&acc)[NQ][4], int lane,
                                            float resc = 1.f) {
  constexpr int TS = (EX & 2) ? 0 : 1;
#pragma unroll
  for (int q = 0; q < NQ; ++q)
#pragma unroll
    for (int cb = 0; cb < 4; ++cb) acc[q][cb] = floatx4{0.f, 0.f, 0.f, 0.f};
  const int boff = h_boff(lane);
  const _Float16* Bh = Hh + boff;
  const _Float16* Bl = Hl + boff;
  half8 ah0[NQ], al0[NQ], ah1[NQ], al1[NQ], bh0[4], bl0[4], bh1[4], bl1[4];
  load_a0<NQ>(A, T, ah0, al0, lane);
#pragma unroll
  for (int cb = 0; cb < 4; ++cb) {
    bh0[cb] = *reinterpret_cast<const half8*>(Bh + cb * 16 * PH);
    bl0[cb] = *reinterpret_cast<const half8*>(Bl + cb * 16 * PH);
  }
  for (int t = 0; t < T; t += 2) {
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      ah1[q] = A[((q * T + TS * (t + 1)) * 2 + 0) * 64 + lane];
      al1[q] = A[((q * T + TS * (t + 1)) * 2 + 1) * 64 + lane];
    }
#pragma unroll
    for (int cb = 0; cb < 4; ++cb) {
      bh1[cb] = *reinterpret_cast<const half8*>(Bh + cb * 16 * PH + 32 * (t + 1));
      bl1[cb] = *reinterpret_cast<const half8*>(Bl + cb * 16 * PH + 32 * (t + 1));
    }
    if (t == 8 && resc != 1.f) rescale_acc<NQ>(acc, resc);
    mfma3_step<PRIO, NQ, EX, LS>(ah0, al0, bh0, bl0, acc);
    const int tn = (t + 2 < T) ? t + 2 : T - 1;
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      ah0[q] = A[((q * T + TS * tn) * 2 + 0) * 64 + lane];
      al0[q] = A[((q * T + TS * tn) * 2 + 1) * 64 + lane];
    }
#pragma unroll
    for (int cb = 0; cb < 4; ++cb) {
      bh0[cb] = *reinterpret_cast<const half8*>(Bh + cb * 16 * PH + 32 * tn);
      bl0[cb] = *reinterpret_cast<const half8*>(Bl + cb * 16 * PH + 32 * tn);
    }
    mfma3_step<PRIO, NQ, EX, LS>(ah1, al1, bh1, bl1, acc);
  }
}

// Ring schedule of the split GEMM (cf. gemm_lite in dsr_mlp_lite.hpp): NB k steps of (hi, lo)
// A fragments in flight through buffer loads (one wave-uniform descriptor, lane offset in one
// VGPR, (q, k step, piece) offset in an SGPR), the (hi, lo) B pair of the next column block
// read from LDS as the current block's MFMAs issue, and the three products of an accumulator
// issued back to back in mfma3_step's order (al.bh, ah.bl, ah.bh) — so the sums are bitwise
// those of gemm16_tile.  The first step starts from an inline zero C operand.
template <bool PRIO, int T, int NB, int LS = 0>
__device__ __forceinline__ void gemm16_ring(const _Float16* Wl, int w, const _Float16* Hh, const _Float16* Hl,
                                            floatx4 (&acc)[4][4], int lane, float resc) {
  const _Float16* base = Wl + (size_t)(4 * w) * T * 2 * 64 * 8;
  const __amdgpu_buffer_rsrc_t rsrc =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<_Float16*>(base), 0, 4 * T * 2 * 1024, 0x00020000);
  const int voff = lane * 16;
  const int boff = h_boff(lane);
  const _Float16* Bh = Hh + boff;
  const _Float16* Bl = Hl + boff;
  auto lda = [&](int q, int t, int piece) {
#ifdef DSR_EXP_NOSTREAM            // timing experiment (invalid results): A from one k step only
    t = 0;
#endif
    return __builtin_bit_cast(
        half8, __builtin_amdgcn_raw_buffer_load_b128(rsrc, voff, ((q * T + t) * 2 + piece) * 1024, 0));
  };
  half8 ah[NB][4], al[NB][4], bh[2], bl[2];
  floatx4 lacc[4][4];                  // LS 2: the lo products' own accumulators
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int cb = 0; cb < 4; ++cb) lacc[q][cb] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int j = 0; j < NB - 1; ++j)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      ah[j][q] = lda(q, j, 0);
      al[j][q] = lda(q, j, 1);
    }
  bh[0] = *reinterpret_cast<const half8*>(Bh);
  bl[0] = *reinterpret_cast<const half8*>(Bl);
  auto step = [&](auto J, auto FIRST, int t) {
    constexpr int j = decltype(J)::value;
    if (t + NB - 1 < T) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        ah[(j + NB - 1) % NB][q] = lda(q, t + NB - 1, 0);
        al[(j + NB - 1) % NB][q] = lda(q, t + NB - 1, 1);
      }
    }
    if (!decltype(FIRST)::value && t == 8 && resc != 1.f) {
      rescale_acc<4>(acc, resc);
      if constexpr (LS == 2) rescale_acc<4>(lacc, resc);
    }
    if (PRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int cb = 0; cb < 4; ++cb) {
      // next B pair: block cb+1 of this step, or block 0 of the next one (after the last step
      // columns 512.. of the 528 pitch / the next point row: in bounds, unused)
      const int nk = (cb < 3) ? (cb + 1) * 16 * PH + 32 * t : 32 * (t + 1);
      bh[(cb + 1) & 1] = *reinterpret_cast<const half8*>(Bh + nk);
      bl[(cb + 1) & 1] = *reinterpret_cast<const half8*>(Bl + nk);
      // keep the next block's B reads here, 12 MFMAs ahead of their use: left to itself the
      // compiler sinks them next to those MFMAs and waits with lgkmcnt(0), exposing the LDS
      // latency whenever the partner wave is not issuing (measured: Jacobian 2.065 -> 2.021 ms
      // per launch, bench +0.9%, bitwise equal; the lite kernel's deeper pinned ring was slower)
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        floatx4 x = decltype(FIRST)::value ? floatx4{0.f, 0.f, 0.f, 0.f} : acc[q][cb];
        if constexpr (LS == 2) {
          lacc[q][cb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al[j][q], bh[cb & 1], lacc[q][cb], 0, 0, 0);
          lacc[q][cb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[j][q], bl[cb & 1], lacc[q][cb], 0, 0, 0);
          acc[q][cb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[j][q], bh[cb & 1], x, 0, 0, 0);
          continue;
        }
        if constexpr (LS == 1) continue;         // below, the block's four q at once
#ifndef DSR_EXP_ONEPROD            // timing experiment (invalid results): the hi.hi product only
        x = __builtin_amdgcn_mfma_f32_16x16x32_f16(al[j][q], bh[cb & 1], x, 0, 0, 0);
        x = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[j][q], bl[cb & 1], x, 0, 0, 0);
#endif
        acc[q][cb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[j][q], bh[cb & 1], x, 0, 0, 0);
      }
      if constexpr (LS == 1) {
        // the four lo chains side by side, the hi products onto the running sums, then the VALU
        // adds of the lo sums
        floatx4 lo[4];
#pragma unroll
        for (int q = 0; q < 4; ++q)
          lo[q] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al[j][q], bh[cb & 1], floatx4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
#pragma unroll
        for (int q = 0; q < 4; ++q) lo[q] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[j][q], bl[cb & 1], lo[q], 0, 0, 0);
#pragma unroll
        for (int q = 0; q < 4; ++q)
          acc[q][cb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(
              ah[j][q], bh[cb & 1], decltype(FIRST)::value ? floatx4{0.f, 0.f, 0.f, 0.f} : acc[q][cb], 0, 0, 0) + lo[q];
      }
    }
    if (PRIO) __builtin_amdgcn_s_setprio(0);
  };
  step(std::integral_constant<int, 0>{}, std::true_type{}, 0);
  constexpr int TM = 1 + (T - 1) / NB * NB;
#pragma unroll 1
  for (int t0 = 1; t0 < TM; t0 += NB) {
    [&]<int... J>(std::integer_sequence<int, J...>) {
      (step(std::integral_constant<int, (1 + J) % NB>{}, std::false_type{}, t0 + J), ...);
    }(std::make_integer_sequence<int, NB>{});
  }
  [&]<int... J>(std::integer_sequence<int, J...>) {
    (step(std::integral_constant<int, (TM + J) % NB>{}, std::false_type{}, TM + J), ...);
  }(std::make_integer_sequence<int, T - TM>{});
  if constexpr (LS == 2) {
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int cb = 0; cb < 4; ++cb) acc[q][cb] += lacc[q][cb];
  }
}

// acc = split product of the wave's 64 rows of packed matrix Wl (K = 32 T, T 16 or 14) and
// the 64-point image: ring schedule with NB k steps in flight (NB 0: gemm16_tile).  `resc`
// (a power of two) moves the partial sums from the image's group-A scale to its group-B
// scale before k step 8 (Scales2); 1 for an image under one scale.
template <bool PRIO, int NB, int LS = 0>
__device__ __forceinline__ void gemm16_sel(const _Float16* Wl, int w, int T, const _Float16* Hh,
                                           const _Float16* Hl, floatx4 (&acc)[4][4], int lane,
                                           float resc = 1.f) {
  if constexpr (NB == 0) {
    gemm16_tile<PRIO, 4, 0, (LS != 0)>(wfrag(Wl, w, T), T, Hh, Hl, acc, lane, resc);
  } else {
    if (T != 14) gemm16_ring<PRIO, 16, NB, LS>(Wl, w, Hh, Hl, acc, lane, resc);
    else gemm16_ring<PRIO, 14, NB, LS>(Wl, w, Hh, Hl, acc, lane, resc);
  }
}

// Every forward and backward split GEMM keeps its lo products in their own accumulators (LS 2).
// The chain must be the same in every kernel that forwards a point: a sample's masks and sdf are
// the same bits whichever kernel computes them (test_gpu_parity.py: the lite pass against the
// exact decode, the broken-block fallback, the surface forward of small batches;
// test_gpu_bench.py: 8-rank shards against one rank).
#if defined(DSR_EXP_JFLS0)
constexpr int JFWD_LS = 0;
#elif defined(DSR_EXP_JFLS1)
constexpr int JFWD_LS = 1;
#else
constexpr int JFWD_LS = 2;
#endif
// the exact pass's surface tiles run the Jacobian kernel's forward chain (the same one unless an
// A/B build sets them apart)
constexpr int SURF_LS = JFWD_LS;
#if defined(DSR_EXP_FLS0)
constexpr int FWD_LS = 0;
#elif defined(DSR_EXP_FLS1)
constexpr int FWD_LS = 1;
#else
constexpr int FWD_LS = 2;
#endif

// power-of-two scale exponent s such that m * 2^s < 2^14 (m >= 0); 0 for m == 0 / non-finite
__device__ __forceinline__ int act_scale_exp(float m) {
  if (!(m > 0.f) || !(m < 3.0e38f)) return 0;
  int e;
  (void)frexpf(m, &e);               // m = f 2^e, f in [0.5, 1)
  return min(14 - e, 126);           // (a tile whose activations all stay below 2^-112: 2^126)
}

__device__ __forceinline__ float wave_max(float v, int lane) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, xor_lane(v, lane, o));
  return v;
}

// Workgroup max of |v| -> power-of-two scale exponent.  Contains the barrier that
// separates the previous GEMM's reads of the image from the writes of the next one.
__device__ __forceinline__ int block_scale(float m, float* wmax, int w, int lane) {
  m = wave_max(m, lane);
  if (lane == 0) wmax[w] = m;
  __syncthreads();
  float mm = wmax[0];
#pragma unroll
  for (int k = 1; k < NWAVE; ++k) mm = fmaxf(mm, wmax[k]);
  return act_scale_exp(mm);
}

// Per-group scales of a forward activation image: rows 0..255 (waves 0-3, the next GEMM's
// k steps 0..7) and rows 256..511 (waves 4-7, k steps 8..15) each from their own group's
// max alone, capped at 2^30 (only an all-tiny group reaches the cap: its values then sit at
// < 2^14 with 11-bit hi pieces and lo pieces down to 2^-27 absolute), so the k-step-8
// rescale 2^(b - a) of the partial sums stays within fp32 for any finite activations below
// 2^90.  Each group can split its rows without the other group's maximum — what a staggered
// schedule needs; here, under the barrier, both are simply read.
__device__ __forceinline__ int group_scale_exp(float m) { return min(act_scale_exp(m), 30); }

struct Scales2 {
  int a, b;
  __device__ __forceinline__ int of(int w) const { return w < 4 ? a : b; }
  __device__ __forceinline__ float resc() const { return ldexpf(1.f, b - a); }
};
__device__ __forceinline__ Scales2 block_scale2(float m, float* wmax, int w, int lane) {
  m = wave_max(m, lane);
  if (lane == 0) wmax[w] = m;
  __syncthreads();
  float ma = wmax[0], mb = wmax[4];
#pragma unroll
  for (int k = 1; k < 4; ++k) {
    ma = fmaxf(ma, wmax[k]);
    mb = fmaxf(mb, wmax[4 + k]);
  }
  return Scales2{group_scale_exp(ma), group_scale_exp(mb)};
}

typedef float float2v __attribute__((ext_vector_type(2)));
typedef _Float16 half2v __attribute__((ext_vector_type(2)));

// Write the wave's 64x64 block of fp32 activations (acc layout, v[q][cb][r]) as hi/lo
// fp16 pieces scaled by 2^s (swizzled image, h_boff).
__device__ __forceinline__ void write_split(const float (&v)[4][4][4], int s, _Float16* Hh, _Float16* Hl,
                                            int w, int lane) {
  const int c = lane & 15, g = (lane >> 4) ^ (((c >> 2) & 1) << 1);
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int n0 = 64 * w + 16 * q + 4 * g;
#pragma unroll
    for (int cb = 0; cb < 4; ++cb) {
      const int p = 16 * cb + c;
      half4 hh, hl;
      // 2^s is a normal float (act_scale_exp keeps s in [-114, 126]): x * 2^s == ldexp(x, s);
      // in pairs (v_pk_mul_f32, v_cvt_pk_f16_f32, v_pk_add_f32)
      const float2v sc2 = float2v{1.f, 1.f} * (ldexpf(1.f, s) * col_sign(cb));   // (col_sign: exact)
#pragma unroll
      for (int r = 0; r < 4; r += 2) {
        const float2v x = float2v{v[q][cb][r], v[q][cb][r + 1]} * sc2;
        const half2v h = __builtin_convertvector(x, half2v);
        hh[r] = h[0]; hh[r + 1] = h[1];
        // lo = fp16(x - h): x - h is exact in fp32, so one fma_mix (f16 operand -h, f32 x,
        // rounded once to f16) per value equals fp16(x - fp32(h)) without the two back-
        // conversions and the subtraction
        const unsigned hb = __builtin_bit_cast(unsigned, h);
        unsigned lb;
        asm("v_fma_mixlo_f16 %0, -%1, 1.0, %2 op_sel_hi:[1,0,0]" : "=v"(lb) : "v"(hb), "v"(x[0]));
        asm("v_fma_mixhi_f16 %0, -%1, 1.0, %2 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "+v"(lb) : "v"(hb), "v"(x[1]));
        const half2v l = __builtin_bit_cast(half2v, lb);
        hl[r] = l[0]; hl[r + 1] = l[1];
      }
      *reinterpret_cast<half4*>(Hh + p * PH + n0) = hh;
      *reinterpret_cast<half4*>(Hl + p * PH + n0) = hl;
    }
  }
}

// Shared epilogue: v = relu(acc * 2^-unscale + bias) (+ xyz rows for lin3), block max,
// one barrier, scale, split-write.  Returns the new activation scale exponent.
// 16-bit lane slices of a layer's ReLU mask (bit (q*4+cb)*4+r of mk, the Jacobian kernel's
// layout) for the lane's 4 points, kept per sample as MaskArgs.msk [point][w][g][layer] (256
// uint16 per point): a lane's 8 layers of one point are 16 contiguous bytes, so the exact
// pass stores them once per tile and the Jacobian kernel loads them with one 16-byte load.
// MaskQueue collects them layer by layer in registers (each push shifts the 8-slot queue by
// one uint16: after layers 0..7, dword k holds layers 2k | 2k+1).
struct MaskQueue {
  unsigned d[4][4];            // [cb][dword]
};

__device__ __forceinline__ void mask_push(MaskQueue& mq, uint64_t mk) {
#pragma unroll
  for (int cb = 0; cb < 4; ++cb) {
    unsigned u = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) u |= (unsigned)((mk >> (16 * q + 4 * cb)) & 0xFull) << (4 * q);
    mq.d[cb][0] = (mq.d[cb][0] >> 16) | (mq.d[cb][1] << 16);
    mq.d[cb][1] = (mq.d[cb][1] >> 16) | (mq.d[cb][2] << 16);
    mq.d[cb][2] = (mq.d[cb][2] >> 16) | (mq.d[cb][3] << 16);
    mq.d[cb][3] = (mq.d[cb][3] >> 16) | (u << 16);
  }
}

__device__ __forceinline__ void mask_store(const MaskQueue& mq, uint16_t* msk, int cand_base, int count, int w,
                                           int lane) {
  const int g = lane >> 4, c = lane & 15;
#pragma unroll
  for (int cb = 0; cb < 4; ++cb) {
    const int p = 16 * cb + c;
    if (p < count)
      *reinterpret_cast<uint4*>(msk + (size_t)(cand_base + p) * 256 + (w * 4 + g) * 8) =
          make_uint4(mq.d[cb][0], mq.d[cb][1], mq.d[cb][2], mq.d[cb][3]);
  }
}

// a if bit I of mask is set, else +0.0: v_bfe_i32 (the bit sign-extended to a 0 / all-ones
// word) + v_and_b32 — bitwise the select `bit ? a : 0.f`, which the compiler otherwise emits
// as and + compare + cndmask (the bit extract is asm so it is not folded back into that)
template <int I>
__device__ __forceinline__ float keep_if(float a, uint64_t mask) {
  const unsigned word = (unsigned)(mask >> (I & 32));
  int m;
  asm("v_bfe_i32 %0, %1, %2, 1" : "=v"(m) : "v"(word), "i"(I & 31));
  return __int_as_float(__float_as_int(a) & m);
}

__device__ __forceinline__ uint64_t relu_bits(const float (&v)[4][4][4]) {
  uint64_t mk = 0;
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int cb = 0; cb < 4; ++cb)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (v[q][cb][r] > 0.f) mk |= 1ull << ((q * 4 + cb) * 4 + r);
  return mk;
}

// lin4's input is h3 | xyz: lin3's padded output rows l3..l3+2 (445..447 at code_len 64: wave 6,
// q 3, g 3, r 1..3; 477..479 at 32: wave 7, q 1) carry the point's x, y, z.  Called under a
// wave-uniform branch (w == l3 >> 6) with the wave-uniform block xq; the row choice is a per-lane
// select, not a per-element divergent branch.  m takes their magnitudes.
template <int NCB>
__device__ __forceinline__ void xyz_rows(float (&v)[4][NCB][4], const float* xyz, int lane, float& m, int xq) {
  const int g = lane >> 4, c = lane & 15;
#pragma unroll
  for (int q = 0; q < 4; ++q) {               // the xyz rows' 16-row block: a wave-uniform choice
    if (q != xq) continue;
    const bool on = g == 3;
#pragma unroll
    for (int cb = 0; cb < NCB; ++cb) {
      const float4 p = *reinterpret_cast<const float4*>(xyz + (16 * cb + c) * 4);
      v[q][cb][1] = on ? p.x : v[q][cb][1];
      v[q][cb][2] = on ? p.y : v[q][cb][2];
      v[q][cb][3] = on ? p.z : v[q][cb][3];
      m = fmaxf(m, on ? fmaxf(fabsf(p.x), fmaxf(fabsf(p.y), fabsf(p.z))) : 0.f);
    }
  }
}

// ---- LayerNorm (deep_sdf_decoder.py:58-63, :96-102: nn.LayerNorm(D) between lin_j and its ReLU,
// eps 1e-5, biased variance) over the D live rows of a layer's pre-activations v (acc layout:
// rows 64w + 16q + 4g + r, points 16cb + c).  The rows of a point span the 8 waves, so the
// per-point moments go through LDS (red / red2, two barriers: mean, then the variance about it —
// two-pass, as torch's LayerNorm accumulates).  Called by all waves.
__device__ __forceinline__ void ln_point_sums(float (&s)[4], float* red, int w, int lane) {
  const int g = lane >> 4, c = lane & 15;
#pragma unroll
  for (int cb = 0; cb < 4; ++cb) {
    s[cb] += xor_lane(s[cb], lane, 16);
    s[cb] += xor_lane(s[cb], lane, 32);
    if (g == 0) red[w * 64 + 16 * cb + c] = s[cb];
  }
}
__device__ __forceinline__ float ln_total(const float* red, int cb, int c) {
  float t = red[16 * cb + c];
#pragma unroll
  for (int k = 1; k < NWAVE; ++k) t += red[k * 64 + 16 * cb + c];
  return t;
}

// v: pre-activations in, u = x^ gamma + beta out (rows >= D: 0).  xh (nullable): the workgroup's
// workspace for this layer (LN_WS_LAYER floats): x^ and rstd are kept for the Jacobian's backward.
__device__ __forceinline__ void ln_fwd(float (&v)[4][4][4], const float* __restrict__ gam,
                                       const float* __restrict__ bet, int D, float* red, float* red2, int w,
                                       int lane, float* __restrict__ xh) {
  const int g = lane >> 4, c = lane & 15;
  float s[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int cb = 0; cb < 4; ++cb)
#pragma unroll
      for (int r = 0; r < 4; ++r) s[cb] += (64 * w + 16 * q + 4 * g + r < D) ? v[q][cb][r] : 0.f;
  ln_point_sums(s, red, w, lane);
  __syncthreads();
  const float invD = 1.f / (float)D;
  float mean[4];
#pragma unroll
  for (int cb = 0; cb < 4; ++cb) {
    mean[cb] = ln_total(red, cb, c) * invD;
    s[cb] = 0.f;
  }
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int cb = 0; cb < 4; ++cb)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float d = v[q][cb][r] - mean[cb];
        s[cb] += (64 * w + 16 * q + 4 * g + r < D) ? d * d : 0.f;
      }
  ln_point_sums(s, red2, w, lane);
  __syncthreads();
  float rstd[4];
#pragma unroll
  for (int cb = 0; cb < 4; ++cb) rstd[cb] = 1.f / sqrtf(ln_total(red2, cb, c) * invD + 1e-5f);
  const int tid = w * 64 + lane;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int n0 = 64 * w + 16 * q + 4 * g;
    const float4 gg = *reinterpret_cast<const float4*>(gam + n0);
    const float4 bb = *reinterpret_cast<const float4*>(bet + n0);
#pragma unroll
    for (int cb = 0; cb < 4; ++cb) {
      float xa[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const bool live = n0 + r < D;
        xa[r] = live ? (v[q][cb][r] - mean[cb]) * rstd[cb] : 0.f;
        v[q][cb][r] = live ? xa[r] * fetch4(gg, r) + fetch4(bb, r) : 0.f;
      }
      if (xh)
        *reinterpret_cast<float4*>(xh + (size_t)((q * 4 + cb) * 512 + tid) * 4) = make_float4(xa[0], xa[1], xa[2], xa[3]);
    }
  }
  if (xh && w == 0 && g == 0) {
#pragma unroll
    for (int cb = 0; cb < 4; ++cb) xh[16 * 512 * 4 + 16 * cb + c] = rstd[cb];
  }
}

// v: dL/du of a LayerNorm layer's output (its ReLU already applied) in, dL/da out:
// rstd (g - mean(g) - x^ mean(g x^)) with g = v gamma, over the D live rows (rows >= D: 0).
// Returns the wave's max |dL/da| (the backward's split scale).
__device__ __forceinline__ float ln_bwd(float (&v)[4][4][4], const float* __restrict__ gam, int D, float* red,
                                        float* red2, int w, int lane, const float* __restrict__ xh) {
  const int g = lane >> 4, c = lane & 15;
  const int tid = w * 64 + lane;
  float s1[4] = {0.f, 0.f, 0.f, 0.f}, s2[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int n0 = 64 * w + 16 * q + 4 * g;
    const float4 gg = *reinterpret_cast<const float4*>(gam + n0);
#pragma unroll
    for (int cb = 0; cb < 4; ++cb) {
      const float4 x4 = *reinterpret_cast<const float4*>(xh + (size_t)((q * 4 + cb) * 512 + tid) * 4);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float gx = (n0 + r < D) ? v[q][cb][r] * fetch4(gg, r) : 0.f;
        s1[cb] += gx;
        s2[cb] += gx * fetch4(x4, r);
      }
    }
  }
  ln_point_sums(s1, red, w, lane);
  ln_point_sums(s2, red2, w, lane);
  __syncthreads();
  const float invD = 1.f / (float)D;
  float m1[4], m2[4], rs[4];
#pragma unroll
  for (int cb = 0; cb < 4; ++cb) {
    m1[cb] = ln_total(red, cb, c) * invD;
    m2[cb] = ln_total(red2, cb, c) * invD;
    rs[cb] = xh[16 * 512 * 4 + 16 * cb + c];
  }
  float m = 0.f;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int n0 = 64 * w + 16 * q + 4 * g;
    const float4 gg = *reinterpret_cast<const float4*>(gam + n0);
#pragma unroll
    for (int cb = 0; cb < 4; ++cb) {
      const float4 x4 = *reinterpret_cast<const float4*>(xh + (size_t)((q * 4 + cb) * 512 + tid) * 4);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const bool live = n0 + r < D;
        const float gx = v[q][cb][r] * fetch4(gg, r);
        const float ga = live ? rs[cb] * ((gx - m1[cb]) - fetch4(x4, r) * m2[cb]) : 0.f;
        v[q][cb][r] = ga;
        m = fmaxf(m, fabsf(ga));
      }
    }
  }
  return m;
}

// LayerNorm after lin7, in place on the unscaled accumulators: acc <- LN(acc + b7); the lin8
// dot then runs on them without the bias (epi_l7 with_bias = false).  xh: as ln_fwd.
__device__ __forceinline__ void ln_l7(floatx4 (&acc)[4][4], const DevDecoder& D, float* red, float* red2, int w,
                                      int lane, float* __restrict__ xh) {
  float (&v)[4][4][4] = reinterpret_cast<float (&)[4][4][4]>(acc);
  const int g = lane >> 4;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const float4 bb = *reinterpret_cast<const float4*>(D.bias[7] + 64 * w + 16 * q + 4 * g);
#pragma unroll
    for (int cb = 0; cb < 4; ++cb)
#pragma unroll
      for (int r = 0; r < 4; ++r) v[q][cb][r] = v[q][cb][r] + fetch4(bb, r);
  }
  ln_fwd(v, D.ln_g[7], D.ln_b[7], D.ln_dim[7], red, red2, w, lane, xh);
}

struct NoStamp {
  __device__ __forceinline__ void operator()(int) const {}
};

// `stamp(phase)` marks phase ends for the DSR_EXP_STAMP diagnostic build (k_mlp_fwd16)
template <class Stamp = NoStamp>
__device__ __forceinline__ Scales2 epi16(floatx4 (&acc)[4][4], int unscale, const float* __restrict__ bias,
                                         Fwd16Shared& sm, int w, int lane, uint64_t& mk, int xr,
                                         Stamp stamp = Stamp{}, const DevDecoder* lnd = nullptr, int l = 0) {
  const int g = lane >> 4, c = lane & 15;
  const float usc = ldexpf(1.f, -unscale);
  float v[4][4][4];
  float m = 0.f;
  uint64_t bits = 0;
  if (lnd != nullptr && ((lnd->ln_mask >> l) & 1)) {   // LayerNorm between lin_l and its ReLU
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float4 bb = *reinterpret_cast<const float4*>(bias + 64 * w + 16 * q + 4 * g);
#pragma unroll
      for (int cb = 0; cb < 4; ++cb)
#pragma unroll
        for (int r = 0; r < 4; ++r) v[q][cb][r] = __builtin_fmaf(accr(acc[q][cb], r), usc * rc_sign(q, cb), fetch4(bb, r));
    }
    ln_fwd(v, lnd->ln_g[l], lnd->ln_b[l], lnd->ln_dim[l], sm.red, sm.red2, w, lane, nullptr);
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int cb = 0; cb < 4; ++cb)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float x = fmaxf(v[q][cb][r], 0.f);
          if (x > 0.f) bits |= 1ull << ((q * 4 + cb) * 4 + r);
          v[q][cb][r] = x;
          m = fmaxf(m, x);
        }
  } else {
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int n0 = 64 * w + 16 * q + 4 * g;
    const float4 bb = *reinterpret_cast<const float4*>(bias + n0);
#pragma unroll
    for (int cb = 0; cb < 4; ++cb) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        // acc*2^-unscale is exact, so the fma rounds exactly like (acc*2^-un) + b; ReLU as
        // v_max (NaN inputs are re-imposed on the output, see nan_in below)
        const float x = fmaxf(__builtin_fmaf(accr(acc[q][cb], r), usc * rc_sign(q, cb), fetch4(bb, r)), 0.f);
        if (x > 0.f) bits |= 1ull << ((q * 4 + cb) * 4 + r);
        v[q][cb][r] = x;
        m = fmaxf(m, x);
      }
    }
  }
  }
  // the next layer's input rows xr..xr+2 <- x, y, z (xyz_row: lin4's input, or every layer's
  // under xyz_in_all); the mask bits above are the ReLU's, taken before
  if (xr >= 0 && w == (xr >> 6)) xyz_rows(v, sm.xyz, lane, m, (xr >> 4) & 3);
  stamp(2);
  const Scales2 sc = block_scale2(m, sm.wmax, w, lane);   // all waves done reading H
  stamp(3);
  write_split(v, sc.of(w), sm.Hh, sm.Hl, w, lane);
  stamp(4);
  mk = bits;
  return sc;
}

// X: bit9 (512) exact re-decode of lite band samples — keep their ReLU masks + sdf
// (MaskArgs); bits 10-11 = NB - 1 of the ring GEMM (gemm16_sel; 0 = the two-set gemm16_tile).
// X bit13 (8192): the decoder-variant instantiation (use_tanh / xyz_in_all / LayerNorm)
template <bool PRIO, int X>
__global__ __launch_bounds__(512) void k_mlp_fwd16(DevDecoder D, const Tile* __restrict__ tiles,
                                                   const int* __restrict__ n_tiles,
                                                   const ObjDesc* __restrict__ desc,
                                                   const float4* __restrict__ cand,
                                                   const float* __restrict__ bias0f,
                                                   const float* __restrict__ bias4f,
                                                   float* __restrict__ dense, unsigned* __restrict__,
                                                   ErtArgs E, MaskArgs MA) {
  __shared__ Fwd16Shared sm;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int nt = *n_tiles;
  constexpr bool MSK = (X & 512) != 0;
  constexpr bool VAR = (X & 8192) != 0;
  constexpr int NB = ((X >> 10) & 3) == 0 ? 0 : 1 + ((X >> 10) & 3);
#ifdef DSR_EXP_STAMP   // diagnostic build: per-wave cycles by phase (as k_mlp_jac16's JSTAMP)
  unsigned long long fst[12] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  unsigned long long fst_last = __builtin_amdgcn_s_memtime();
  int ftiles = 0;
  auto stamp = [&](int cat) {
    __builtin_amdgcn_sched_barrier(0);
    const unsigned long long t = __builtin_amdgcn_s_memtime();
    fst[cat] += t - fst_last;
    fst_last = t;
    __builtin_amdgcn_sched_barrier(0);
  };
#else
  NoStamp stamp;
#endif
  for (int ti = blockIdx.x; ti < nt; ti += gridDim.x) {
#ifdef DSR_EXP_STAMP
    ++ftiles;
#endif
    const Tile tl = tiles[ti];
    const ObjDesc d = desc[tl.obj];
    // term 3 (MSK): surface points, object frame as in the Jacobian kernel; their masks and
    // sdf go to the surface slots, nothing else is written for them
    const bool surf = MSK && tl.term == 3;
    const int mbase = surf ? MA.surf_base + d.pts_off + tl.start : d.cand_off + tl.start;
    // wave 0 (point tid = lane) also fetches what the tile's tail reads from global memory —
    // the code's NaN probe and the sample's lite value — so those loads are in flight
    // during the layers instead of exposed in the tail, where the other waves wait for it
    float zpre = 0.f, ylpre = 0.f;
    {
      const int tid = opaque(threadIdx.x);
      if (tid < TILE) {
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        zpre = bias0f[tl.obj * HID];
        if (tid < tl.count) {
          if (surf) {
            const float* p = MA.pts + (size_t)(d.pts_off + tl.start + tid) * 3;
            const float3 xo = xform(E.st[tl.obj].T, p[0], p[1], p[2]);
            v = make_float4(xo.x, xo.y, xo.z, 0.f);
          } else {
            v = cand[d.cand_off + tl.start + tid];
            if (E.st) ylpre = dense[d.cand_off + (__float_as_int(v.w) & ~AUDIT_BIT)];
          }
        }
        *reinterpret_cast<float4*>(sm.xyz + tid * 4) = v;
      }
    }
    __syncthreads();
    stamp(0);
    // ---- lin0 on VALU (fp32), then split
    Scales2 sa;
    MaskQueue mq;
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
          const float4 p = *reinterpret_cast<const float4*>(sm.xyz + (16 * cb + c) * 4);
#pragma unroll
          for (int r = 0; r < 4; ++r)
            v[q][cb][r] = fetch4(bb, r) + ((wx[3 * r] * p.x + wx[3 * r + 1] * p.y) + wx[3 * r + 2] * p.z);
        }
      }
      if (VAR && (D.ln_mask & 1)) ln_fwd(v, D.ln_g[0], D.ln_b[0], D.ln_dim[0], sm.red, sm.red2, w, lane, nullptr);
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int cb = 0; cb < 4; ++cb)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            v[q][cb][r] = fmaxf(v[q][cb][r], 0.f);
            m = fmaxf(m, v[q][cb][r]);
          }
      uint64_t b0 = 0;
      if constexpr (MSK) b0 = relu_bits(v);
      if (VAR && D.xyz_all && w == 7) xyz_rows(v, sm.xyz, lane, m, 3);   // lin1's input = h0 | xyz
      sa = block_scale2(m, sm.wmax, w, lane);
      write_split(v, sa.of(w), sm.Hh, sm.Hl, w, lane);
      if constexpr (MSK) mask_push(mq, b0);
    }
    __syncthreads();
    floatx4 acc[4][4];
#pragma unroll 1
    for (int l = 1; l <= 6; ++l) {
      const int lane = opaque(threadIdx.x & 63);
      stamp(7);
      if (SURF_LS != FWD_LS && surf) gemm16_sel<PRIO, NB, SURF_LS>(D.Wh_raw[l], w, D.Kf[l] / 32, sm.Hh, sm.Hl, acc, lane, sa.resc());
      else gemm16_sel<PRIO, NB, FWD_LS>(D.Wh_raw[l], w, D.Kf[l] / 32, sm.Hh, sm.Hl, acc, lane, sa.resc());
      stamp(1);
      uint64_t mk;
      sa = epi16(acc, D.sw[l] + sa.b, (l == 4) ? bias4f + tl.obj * HID : D.bias[l], sm, w, lane, mk,
                 VAR ? xyz_row(D, l) : (l == 3 ? D.l3 : -1), stamp, VAR ? &D : nullptr, l);
      if constexpr (MSK) mask_push(mq, mk);
      stamp(7);
      __syncthreads();
      stamp(5);
    }
    {
      const int lane = opaque(threadIdx.x & 63);
      stamp(7);
      if (SURF_LS != FWD_LS && surf) gemm16_sel<PRIO, NB, SURF_LS>(D.Wh_raw[7], w, D.Kf[7] / 32, sm.Hh, sm.Hl, acc, lane, sa.resc());
      else gemm16_sel<PRIO, NB, FWD_LS>(D.Wh_raw[7], w, D.Kf[7] / 32, sm.Hh, sm.Hl, acc, lane, sa.resc());
      stamp(1);
      const int un = D.sw[7] + sa.b;
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int cb = 0; cb < 4; ++cb)
#pragma unroll
          for (int r = 0; r < 4; ++r) acc[q][cb][r] = ldexpf(acc[q][cb][r], -un) * rc_sign(q, cb);
      uint64_t mask;
      const bool ln7 = VAR && ((D.ln_mask >> 7) & 1);
      if (ln7) ln_l7(acc, D, sm.red, sm.red2, w, lane, nullptr);
      epi_l7(acc, D, sm.red, w, lane, mask, VAR ? sm.xyz : nullptr, !ln7);
      if constexpr (MSK) {
        mask_push(mq, mask);
        mask_store(mq, MA.msk, mbase, tl.count, w, lane);
      }
      stamp(8);
    }
    __syncthreads();
    stamp(9);
    {
      const int tid = opaque(threadIdx.x);
      float emax = 0.f;
      if (tid < tl.count) {
        float s = sm.red[tid];
        for (int k = 1; k < NWAVE; ++k) s += sm.red[k * TILE + tid];
        float y = tanhf(s + D.b8);
        if (VAR && D.use_tanh) y = tanhf(y);           // use_tanh: lin8 -> tanh -> self.th
        stamp(10);
        // the ReLUs above are v_max (NaN -> 0); torch.relu propagates NaN, and a NaN can only
        // enter through the point or the code, so re-impose it here
        const float4 p = *reinterpret_cast<const float4*>(sm.xyz + tid * 4);
        const float zprobe = zpre;                     // NaN iff the code holds a NaN
        if (p.x != p.x || p.y != p.y || p.z != p.z || zprobe != zprobe) y = __builtin_nanf("");
        if (surf) {
          MA.yv[mbase + tid] = y;
        } else {
          const int tagged = __float_as_int(p.w);
          const int idx = tagged & ~AUDIT_BIT;
          if (E.st) {                      // re-decode after the lite pass: track the lite error
            const float yl = ylpre;
            const float e = fabsf(y - yl);
            if (e == e) emax = e;
            if (tagged & AUDIT_BIT) {      // audited out-of-band sample: same class exactly?
              const int cl = yl <= E.nth ? 0 : (yl < -E.nth ? 1 : 2);   // full | band | empty
              const int ce = y <= E.nth ? 0 : (y < -E.nth ? 1 : 2);
              if (cl != ce) atomicAdd(&E.st[tl.obj].lite_viol, 1);
            }
          }
          dense[d.cand_off + idx] = y;
          if constexpr (MSK) MA.yv[d.cand_off + tl.start + tid] = y;
          if (E.dead && y <= E.nth) dead_put(E.dead + d.ray_off + idx / E.M, 1);   // occupancy 1: ray terminated
        }
      }
      stamp(11);
      // the tile's largest |lite - exact|: one atomic per tile instead of one per sample
      if (w == 0 && E.st && !surf) {
        emax = wave_max(emax, opaque(threadIdx.x & 63));
        if ((threadIdx.x & 63) == 0 && emax > 0.f)
          atomicMax(reinterpret_cast<int*>(&E.st[tl.obj].lite_err), __float_as_int(emax));
      }
    }
    __syncthreads();
    stamp(6);
  }
#ifdef DSR_EXP_STAMP
  if (blockIdx.x < 4 && (threadIdx.x == 0 || threadIdx.x == 256))
    printf("fwd16_stamp %d %d %d %llu %llu %llu %llu %llu %llu %llu %llu %llu %llu %llu %llu\n", (int)blockIdx.x, w,
           ftiles, fst[0], fst[1], fst[2], fst[3], fst[4], fst[5], fst[6], fst[7], fst[8], fst[9], fst[10], fst[11]);
#endif
}

}  // namespace dsr

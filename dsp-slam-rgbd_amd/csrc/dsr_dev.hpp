// dsr_dev.hpp — device-side data layout shared by all libdsr kernels.
//
// Data layout in HBM (one batch of n_obj objects):
//   pts   [sum n_pts][3]    surface points, camera frame          (input, resident)
//   rays  [sum n_rays][3]   ray directions, fg first              (input, resident)
//   dobs  [sum n_rays]      observed depth (fg) / 1.1*d_max (bg)   (input + per-iter)
//   cand  [sum n_rays*M]    float4 (x,y,z, bits(ray*M+j)): ray samples inside the unit
//                           ball, compacted in (ray, depth) order == torch.where order
//   dense [sum n_rays*M]    SDF per (ray, depth) sample, NaN when outside the ball
//   kpts  [sum n_rays*M]    float4 (x,y,z, de_ds) of the K render points
//   kres  [sum n_rays*M]    clamped depth residual of the K render points
//   slots [n_jac_tiles][SLOT_FLOATS] per-tile partial J^T J (upper tri), J^T r~, sum r~^2
// Decoder weights are packed once into MFMA A-fragment order (see pack_frag in
// dsr_api.hip) so each wave-instruction of a weight load reads 1 KiB contiguous.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dsr {

constexpr int HID = 512;          // hidden width (dims=[512]*8)
constexpr int CODE = 64;          // code_len
constexpr int IN = CODE + 3;      // decoder input width
constexpr int NPOSE = 7;          // Sim(3) tangent: rho(3) omega(3) s
constexpr int NPAR = NPOSE + CODE;   // 71
constexpr int NTRI = NPAR * (NPAR + 1) / 2;   // 2556 upper-triangle entries
constexpr int SLOT_FLOATS = NTRI + NPAR + 1;  // + J^T r~ (71) + sum r~^2
constexpr int TILE = 64;          // points per MLP tile
constexpr int PITCH = 520;        // LDS row pitch (floats) of the [point][neuron] image:
                                  // conflict-free ds_read_b128 for the B-fragment reads
constexpr int NWAVE = 8;          // waves per MLP workgroup (512 threads)
constexpr int MAXM = 64;          // max depth samples per ray
constexpr int L3_OUT = 445;       // lin3 out (= 512 - 67, latent re-injection)

typedef float floatx4 __attribute__((ext_vector_type(4)));

struct DevDecoder {
  const float4* Wf[8];   // forward A-fragments of lin1..lin7 (index = layer), [32 rb][K/16][64 lanes]
  int Kf[8];             // padded K of each forward layer (512; 448 for lin4 = h3|xyz)
  const float4* Wb[8];   // backward A-fragments of lin_l^T (l=1..7), Wb[0] = lin0^T (80 rows)
  int Kb[8];             // K of each backward GEMM (512; 448 for lin3^T)
  const float* bias[8];  // b_l padded to 512 (l = 0..7)
  const float* W0x;      // [512][3]  lin0 xyz columns
  const float* W0z;      // [64][512] lin0 code columns, k-major (folded into a per-object bias)
  const float* W4z;      // [64][512] lin4 code columns, k-major (folded into a per-object bias)
  const float* W8;       // [512]     lin8 row
  float b8;
  // split-fp16 copies of the forward A-fragments (dsr_mlp16.hpp):
  // [32 rb][K/32][2 pieces (hi, lo)][64 lanes] x 8 halfs, scaled by 2^sw[l]
  const _Float16* Wh_raw[8];
  int sw[8];
  // lite-pass copies (dsr_mlp_lite.hpp, LV bit8): fp16(W) unscaled, hi pieces only,
  // [32 rb][K/32][64 lanes] x 8 halfs
  const _Float16* Wl_raw[8];
  // split-fp16 backward A-fragments of lin_l^T (l = 1..7; [0] = lin0^T, 80 rows), scale 2^swb[l]
  const _Float16* Wbh_raw[8];
  int swb[8];
  // code length (64 or 32; a 32-D decoder runs in the 64-D layout with its code columns 32..63 of
  // lin0 / lin4 zero and its code held at zero there) and lin3's output count l3 = 509 - code_len
  // (445 / 477): lin4's input is [h3 (l3) | code | xyz], so its xyz rows are l3..l3+2 — wave
  // l3 >> 6, 16-row block (l3 >> 4) & 3, quad g = 3, rows r = 1..3 (l3 % 16 == 13 for both)
  int code_len;
  int l3;
  // decoder variants of deep_sdf_decoder.py (split-fp16 kernels only; never lite-eligible):
  // xyz_all (xyz_in_all, :46-47, :89-90): every hidden layer but lin3 has 509 outputs and every
  // layer's input but lin0's / lin4's is [h (509) | xyz] — rows 509..511 (wave 7, block 3, quad
  // 3, r 1..3, like lin4's) carry the point's x, y, z after the ReLU, lin8's included;
  // use_tanh (:65-67, :93-94): tanh after lin8, before the final self.th — y = tanh(tanh(.))
  int xyz_all;
  int use_tanh;
  // LayerNorm (weight_norm=False with norm_layers, deep_sdf_decoder.py:58-63, :96-102): bit j of
  // ln_mask = nn.LayerNorm(out_dim_j) between lin_j and its ReLU (eps 1e-5, biased variance),
  // gamma / beta padded to 512 with zeros, ln_dim[j] = out_dim_j (the rows it normalises over)
  int ln_mask;
  int ln_dim[8];
  const float* ln_g[8];
  const float* ln_b[8];
};

// Per-workgroup workspace of the Jacobian kernel for LayerNorm decoders: each LayerNorm layer's
// normalised activations x^ (acc layout, [16 (q, cb)][512 threads] float4) and rstd per point,
// written by the forward and read back by the backward of the same tile
constexpr int LN_WS_LAYER = 16 * 512 * 4 + 64;     // floats
constexpr int LN_WS_WG = 8 * LN_WS_LAYER;          // floats per workgroup (262,656 floats = 1.05 MB:
                                                   // 8 layers x (16 float4 x 512 threads + rstd)); n_cu
                                                   // of them per stream, so ~270 MB per object-group
                                                   // stream on MI355X's 256 CUs, allocated only for
                                                   // LayerNorm decoders (never DSP-SLAM's)

// row of the point's xyz in the input of the layer after lin_l (l = 0..7), or -1: lin4's input
// is [h3 | code (folded) | xyz] (row l3), with xyz_in_all every other layer's is [h | xyz] (509)
__device__ __forceinline__ int xyz_row(const DevDecoder& D, int l) {
  return l == 3 ? D.l3 : (D.xyz_all ? HID - 3 : -1);
}

// d sdf / d[code, xyz] slot (gin, 64-D layout: code 0..63, xyz 64..66) of lin4's input row n >= l3
__device__ __forceinline__ int gin_slot(int n, int l3) { return n < HID - 3 ? n - l3 : CODE + (n - (HID - 3)); }

// Kernels built without packed-FP32 VALU instructions (v_pk_mul/add/fma_f32): DESIGN.md §3.9.
// DSR_EXP_PKSCAN (diagnostic builds) keeps them, to reproduce the round-6 finding.
#ifdef DSR_EXP_PKSCAN
#define DSR_NO_PK_F32
#else
#define DSR_NO_PK_F32 __attribute__((target("no-packed-fp32-ops")))
#endif

struct ObjDesc {
  int pts_off, n_pts;    // into pts
  int ray_off, n_rays;   // into rays / dobs
  int n_fg;              // foreground rays (have observed depth)
  int cand_off;          // into cand / dense / kpts / kres  (capacity n_rays*M)
  int slot_sdf;          // first jac slot of this object's sdf tiles
  int pad;
};

enum { ST_RUNNING = 0, ST_DONE = 1, ST_FAIL = 2 };

struct ObjState {
  float T[16];           // t_obj_cam (camera -> object), row-major
  float Tco[16];         // inverse(T) of this iteration (optimizer.py:122)
  float depths[MAXM];    // torch.linspace(d_min, d_max, M) (optimizer.py:126)
  float dmin, dmax, delta_d, bg_depth;
  float loss;            // returned loss (pre-update value of the last good iteration)
  float sdf_loss, render_loss;
  int status;            // ST_*
  int fail_reason;       // DSR_FAIL_*
  int iters_done;
  int n_valid, k;        // this iteration's counts
  int n_sdf_tiles, n_ren_tiles, slot_ren;   // this iteration's jac tiles
  int n_emit;            // ray samples emitted by the current render pass (fwd tiles)
  int n_eval;            // ray samples decoded this iteration (sum over passes)
  int n_refine;          // of which re-decoded exactly after the lite pass
  float lite_margin;     // this iteration's classification margin (dsr_mlp_lite.hpp)
  float lite_err;        // max |lite - exact| seen on this object's re-decoded samples
  int n_audit;           // this iteration's audited out-of-band samples (k_refine_scan)
  int lite_viol;         // this iteration's audited samples whose exact class differs
  int lite_viol_total;   // over the run
  int lite_redo;         // 1: an iteration was discarded for a violation; exact from then on
  int pad_[8];           // whole 128 B lines per object: no line holds two groups' objects
};
static_assert(sizeof(ObjState) % 128 == 0, "ObjState spans whole cache lines");

struct Tile {
  int obj, term, start, count;   // term: 0 = sdf (surface points), 1 = render (K list),
                                 // 3 = surface points in the exact pass (MaskArgs.pts)
};

// Early ray termination (k_sample_pass): the fwd kernels flag a ray dead once one of its
// samples decodes to sdf <= -cut_off (occupancy exactly 1, transmittance exactly 0 after it).
// dead-flag accesses (experiment DSR_EXP_DEADWT: system-scope relaxed atomics, i.e. vector
// loads / stores that bypass the non-coherent caches)
__device__ __forceinline__ void dead_put(int* p, int v) {
#ifdef DSR_EXP_DEADWT
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
#else
  *p = v;
#endif
}
__device__ __forceinline__ int dead_get(int* p) {
#ifdef DSR_EXP_DEADWT
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
#else
  return *p;
#endif
}
#ifdef DSR_EXP_PROV
// Diagnostic build only (tools/prov_diff.py): per-run provenance of the early
// ray termination — for every (iteration, pass start rank, ray) whether k_sample_pass found the
// ray alive and how many samples it emitted, for every (iteration, sample) the lite value, and
// for every (iteration, ray) the first depth index whose lite value terminated it.
constexpr int PROV_IT = 12;
__device__ int* g_prov_alive;   // [PROV_IT][64][R]: cnt + 1 (alive), -1 (dead), 0 (not visited)
__device__ float* g_prov_y;     // [PROV_IT][C]: lite value (NaN: not decoded)
__device__ int* g_prov_set;     // [PROV_IT][R]: smallest j that set the dead flag (INT_MAX: none)
__device__ int* g_prov_xcc;     // [PROV_IT][R][2]: XCC of the workgroup that cleared / set the flag
__device__ int* g_prov_j;       // [PROV_IT][64][R]: first depth index emitted by the pass (-1: none)
__device__ unsigned* g_prov_t;  // [PROV_IT][65][R]: s_memrealtime (low 32 bits) of each pass's read
                                // of the flag (rows 0..63) and of the first set (row 64)
__device__ unsigned* g_prov_h;  // [2][PROV_IT][R][3]: (checksum of the object's pose T[0..11] and depths,
                                // s_memrealtime, XCC) as k_iter_begin wrote them (row 0, key: the
                                // object's first ray) and as each k_sample_scan chunk staged them
                                // (row 1, key: the chunk's first ray)
__device__ int g_prov_R, g_prov_C;
__device__ float* g_prov_nrm2;  // [PROV_IT][R][8]: the same check in k_sample_pass's first-pass scan
__device__ float* g_prov_nrm;   // [PROV_IT][R][12]: k_sample_scan's |x| of samples 0..3 in its loop,
                                // recomputed after it, and the LDS depths 0..3 re-read after it
__device__ unsigned* g_prov_ri; // [2][PROV_IT][R][2]: (rinfo value, s_memrealtime) as k_sample_scan wrote it
                                // (row 0) and as the first k_sample_pass read it (row 1)
__device__ inline void prov_rinfo(int row, int it, int ray, int v) {
  if (!g_prov_ri || it >= PROV_IT) return;
  unsigned* p = g_prov_ri + (((size_t)row * PROV_IT + it) * g_prov_R + ray) * 2;
  p[0] = (unsigned)v;
  p[1] = (unsigned)__builtin_amdgcn_s_memrealtime();
}
__device__ inline unsigned prov_sum(const float* T, const float* dep, int M) {
  unsigned h = 0;
  for (int i = 0; i < 12; ++i) h += __float_as_uint(T[i]) * (2u * i + 1u);
  for (int i = 0; i < M; ++i) h += __float_as_uint(dep[i]) * (2u * i + 25u);
  return h;
}
__device__ inline void prov_state(int row, int it, int key, unsigned h) {
  if (!g_prov_h || it >= PROV_IT) return;
  unsigned* p = g_prov_h + (((size_t)row * PROV_IT + it) * g_prov_R + key) * 3;
  p[0] = h;
  p[1] = (unsigned)__builtin_amdgcn_s_memrealtime();
  p[2] = (unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 20);
}
__device__ inline unsigned prov_now() { return (unsigned)__builtin_amdgcn_s_memrealtime(); }
__device__ inline void prov_emit(int it, int ra, int ray, int j) {
  if (!g_prov_j || it >= PROV_IT || ra >= 64) return;
  g_prov_j[((size_t)it * 64 + ra) * g_prov_R + ray] = j;
  g_prov_t[((size_t)it * 65 + ra) * g_prov_R + ray] = prov_now();
}
__device__ inline int prov_xcc() { return (int)__builtin_amdgcn_s_getreg((31 << 11) | 20); }
// alive entries: (cnt + 1 | -1) + 1024 * the reading workgroup's XCC
__device__ inline void prov_alive(int it, int ra, int ray, int v) {
  if (g_prov_alive && it < PROV_IT && ra < 64)
    g_prov_alive[((size_t)it * 64 + ra) * g_prov_R + ray] = v + 1024 * prov_xcc();
}
__device__ inline void prov_clear(int it, int ray) {
  if (g_prov_xcc && it < PROV_IT) g_prov_xcc[((size_t)it * g_prov_R + ray) * 2] = prov_xcc();
}
__device__ inline void prov_lite(int it, int sample, int ray, int j, float y, bool sets_dead) {
  if (!g_prov_y || it >= PROV_IT) return;   // (decoder qualification, sdf queries: no batch)
  g_prov_y[(size_t)it * g_prov_C + sample] = y;
  if (sets_dead) {
    atomicMin(g_prov_set + (size_t)it * g_prov_R + ray, j);
    atomicMin(g_prov_t + ((size_t)it * 65 + 64) * g_prov_R + ray, prov_now());
    g_prov_xcc[((size_t)it * g_prov_R + ray) * 2 + 1] = prov_xcc();
  }
}
#endif
struct ObjState;
struct ErtArgs {
  int* dead;             // [sum n_rays] (nullptr: no flagging, e.g. dsr_sdf_eval)
  int M;                 // samples per ray (grid index = ray * M + j)
  float nth;             // -cut_off
  ObjState* st;          // lite pass: per-object margin; exact re-decode: per-object error
  unsigned char* refine; // lite pass: [sum n_rays*M] samples to decode exactly
  int lag;               // staggered lite pass: k step at which group B may start a GEMM
  // lite-pass audit (dsr_mlp_lite.hpp: lite_flag): out-of-band samples with |y| < th +
  // (1 + shell)*margin — the band edge plus `shell` margins — and a hashed 2^-audit_log2 share
  // of all others (audit_log2 = 0: every sample) are re-decoded exactly too
  int audit;             // 0: no audit
  float shell;
  int audit_log2;
  float perturb;         // test hook (DSR_LITE_PERTURB, only with DSR_TEST_HOOKS=1): lite values moved by +-perturb
  int* diag;             // staggered lite pass: [0] blocks whose event wait expired, [1..] the first
                         // expired wait's record (StDiag, dsr_mlp_lite.hpp); nullptr: none kept
};

// Record of the first expired event wait of a batch run (k_mlp_fwd_lite_st, st_wait), in
// ErtArgs.diag.  Read by dsr_batch_stats (dsr_stats.lite_broken_blocks) and the diagnostics
// entry point dsr_batch_lite_diag.
enum {
  STD_BROKEN = 0,        // blocks that marked themselves broken (all launches of the run)
  STD_CLAIM,             // 1 once the record below is written
  STD_BLOCK, STD_WAVE, STD_COUNTER, STD_TARGET, STD_OBSERVED, STD_IT, STD_HWID, STD_XCC,
  STD_POLLS,             // polls from the clock start (poll 1024) to expiry
  STD_REAL,              // 100 MHz ticks (s_memrealtime) over those polls
  STD_INTS
};

// bit 30 of a refine candidate's sample index (cand[].w): the sample is an audit, not a band sample
constexpr int AUDIT_BIT = 1 << 30;

// Lite-pass classification of one decoded sample (lite value y, index idx = ray*M + j)
// into the refine flags k_refine_scan consumes: 1 = band (|y| < th + margin, NaN, or
// the range guard), 2 = audited certainly-empty sample, 3 = audited certainly-full sample
// (3 also terminates the ray, like an unaudited full sample).  Returns the flag (0: none)
// and sets `full` when the sample is certainly full.
__device__ __forceinline__ unsigned char lite_flag(const ErtArgs& E, float y, int idx, float margin,
                                                   int salt, bool& full) {
  full = false;
  if (!(y >= -E.nth + margin) && !(y <= E.nth - margin)) return 1;      // band (or NaN)
  full = y <= E.nth - margin;
  if (!E.audit) return 0;
  const unsigned h = (unsigned)(idx ^ (salt * 0x5bd1e995)) * 2654435761u;
  const bool au = fabsf(y) < -E.nth + (1.f + E.shell) * margin ||
                  E.audit_log2 == 0 || (h >> (32 - E.audit_log2)) == 0u;
  return au ? (full ? 3 : 2) : 0;
}

// test hook: a deterministic +-perturb on every lite value (DSR_LITE_PERTURB; the library
// honours it only under DSR_TEST_HOOKS=1, which dsr_stats.test_hooks reports)
__device__ __forceinline__ float lite_perturb(const ErtArgs& E, float y, int idx) {
  if (E.perturb == 0.f) return y;
  return y + ((((unsigned)idx * 2654435761u) >> 31) ? E.perturb : -E.perturb);
}

// ReLU masks + SDF of the samples the exact pass re-decodes after the lite pass, so the
// Jacobian kernel runs only the backward chain for render points (loss.py:157 re-forwards
// them through autograd; the masks and tanh input are the same values).
//   msk[slot][layer 0..7][wave 0..7][g 0..3]: 16 bits = rows 64w + 16q + 4g + r (bit 4q+r)
//   yv[slot]: sdf; slotmap[sample] = slot (or -1); kslot[k] = slot of render point k
// (slot, sample and k are offsets from the object's cand_off)
//   Surface points (pts != nullptr): the exact pass also runs the forward of every
//   surface-point tile (Tile.term 3) and keeps its masks + sdf at slot
//   surf_base + pts_off + point, so the Jacobian kernel runs the backward chain only for
//   every tile, sdf and render alike (one weight direction per kernel: half the L2 set).
struct MaskArgs {
  uint16_t* msk;
  float* yv;
  int* slotmap;
  const int* kslot;
  const float* pts;      // surface points (camera frame), or nullptr: the Jacobian forwards them
  int surf_base;         // first mask slot of the surface points
};

struct GNParams {
  float k1, k2, k3, k4, b1, b2, lr, s_damp, cut_off;
  int iters, M;
  int raw_residual;      // 1: J^T r with the un-robustified residual (pose-only GN, optimizer.py:71)
  float lite_margin0;    // lite pass: first-iteration margin
  float lite_floor;      // ... smallest margin
  float lite_safety;     // ... margin = max(floor, safety x max observed lite error)
};

// (p[...,None,:] * T[:3,:3]).sum(-1) + T[:3,3]   (loss.py:31-32, :74-77)
__device__ __forceinline__ float3 xform(const float* T, float x, float y, float z) {
  float3 o;
  o.x = ((x * T[0] + y * T[1]) + z * T[2]) + T[3];
  o.y = ((x * T[4] + y * T[5]) + z * T[6]) + T[7];
  o.z = ((x * T[8] + y * T[9]) + z * T[10]) + T[11];
  return o;
}

__device__ __forceinline__ float fetch4(const float4& v, int j) {
  return j == 0 ? v.x : (j == 1 ? v.y : (j == 2 ? v.z : v.w));
}

// x, re-materialised at this point: the compiler may not assume it equals an earlier x, so
// values derived from it are computed where they are used instead of being hoisted to the
// kernel entry and kept live (or spilled) across every GEMM
__device__ __forceinline__ int opaque(int x) {
  asm volatile("" : "+v"(x));
  return x;
}

// v of lane (lane ^ o): ds_bpermute with an index derived from the caller's (opaque) lane
__device__ __forceinline__ float xor_lane(float v, int lane, int o) {
  return __int_as_float(__builtin_amdgcn_ds_bpermute((lane ^ o) << 2, __float_as_int(v)));
}

}  // namespace dsr

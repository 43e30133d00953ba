/*
 * dsr.h — C ABI of libdsr, the MI355X-native DeepSDF shape-prior reconstruction
 * hot path (DSP-SLAM reconstruct/optimizer.py + loss.py + loss_utils.py +
 * deep_sdf/deep_sdf_decoder.py).
 *
 * The reference exposes this path only as Python (`reconstruct.optimizer.Optimizer`,
 * called from C++ ORB-SLAM2 through pybind11: src/LocalMapping_util.cc:181-182,
 * :394-395, :109-110, src/MapObject_util.cc:43).  The build keeps that Python API
 * (dsp-slam-rgbd_amd/reconstruct) and puts this library underneath it, loaded with
 * ctypes.  Every entry point below names the reference interface it replaces.
 *
 * Conventions
 *   - plain C types only; all matrices are row-major float32 (numpy C order);
 *   - every function returns int status: 0 = ok, <0 = error (message via
 *     dsr_last_error); numeric failure of an object is NOT an error — it is
 *     reported per object in dsr_object_out.is_good (reference convention,
 *     optimizer.py:132-152);
 *   - the caller owns all host buffers for the duration of a call; the library
 *     owns device memory; calls are synchronous unless stated otherwise;
 *   - a context is bound to one HIP device and is not thread-safe (the reference's
 *     callers are serialized on the GIL, include/System.h:57-71).
 */
#ifndef DSR_H
#define DSR_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DSR_ABI_VERSION 11
#define DSR_MAX_LAYERS 16
#define DSR_CODE_LEN 64

typedef struct dsr_ctx dsr_ctx;
typedef struct dsr_decoder dsr_decoder;
typedef struct dsr_batch dsr_batch;

/* Architecture of a DeepSDF decoder (replaces deep_sdf/deep_sdf_decoder.py:10-72 as
 * configured by specs.json through deep_sdf/workspace.py:202-223): dims [512]*8, latent
 * re-injection at lin4, ReLU, final self.th tanh, CodeLength 64 or 32, and the module's
 * use_tanh / xyz_in_all / LayerNorm switches (weight-norm or plain linear layers are folded by
 * the caller).  Anything else is rejected with an error (never silently approximated). */
typedef struct {
  int code_len;                   /* CodeLength (64) */
  int n_layers;                   /* number of lin{i} (9 for dims=[512]*8) */
  int out_dim[DSR_MAX_LAYERS];    /* rows of lin{i}.weight */
  int in_dim[DSR_MAX_LAYERS];     /* cols of lin{i}.weight */
  int latent_in;                  /* index of the layer that takes cat([x, input]) (4) */
  int use_tanh;                   /* NetworkSpecs.use_tanh: tanh after lin8, before the final tanh
                                     (deep_sdf_decoder.py:65-67, 93-94) — 0 or 1 */
  int xyz_in_all;                 /* NetworkSpecs.xyz_in_all (:46-47, 89-90): hidden layers but lin3 have
                                     509 outputs, every layer input but lin0's / lin4's is [h | xyz] — 0 or 1.
                                     Either variant runs the split-fp16 kernels and never the lite pass
                                     (dsr_decoder_info.lite_eligible 0) */
  int norm_mask;                  /* ABI 9: bit j = nn.LayerNorm(out_dim_j) between lin{j} and its ReLU
                                     (weight_norm=False with j in norm_layers, :58-63, 96-102; eps 1e-5).
                                     The weight buffer then continues, for each such j in order, with
                                     bn{j}.weight (gamma, out_dim_j) and bn{j}.bias (beta, out_dim_j).
                                     Split-fp16 kernels only, never the lite pass.  0 for DSP-SLAM's decoders */
} dsr_decoder_desc;

/* Optimizer hyper-parameters (reconstruct/optimizer.py:27-43; configs/config_*.json
 * "optimizer" block). */
typedef struct {
  float k1, k2, k3, k4;           /* render, sdf, code-reg, rotation-prior weights */
  float b1, b2;                   /* Huber thresholds render / sdf */
  float lr;                       /* joint_optim.learning_rate */
  float s_damp;                   /* joint_optim.scale_damping */
  int num_iterations;             /* joint_optim.num_iterations */
  int code_len;                   /* must equal the decoder's code_len */
  int num_depth_samples;          /* M (50), <= 64 */
  float cut_off;                  /* cut_off_threshold (0.01) */
  int pose_only_iterations;       /* pose_only_optim.num_iterations (5) */
} dsr_optim_params;

/* One object handed to Optimizer.reconstruct_object(t_cam_obj, pts, rays, depth,
 * code) — optimizer.py:90. */
typedef struct {
  float t_cam_obj[16];            /* initial object->camera Sim(3), row-major */
  const float* pts;               /* (n_pts,3) surface points, camera frame */
  int n_pts;
  const float* rays;              /* (n_rays,3) ray directions, fg rays first */
  int n_rays;
  const float* depth;             /* (n_depth,) observed depth of the fg rays */
  int n_depth;                    /* n_fg; n_rays - n_depth background rays */
  const float* code;              /* (code_len,) warm-start code or NULL (=zeros) */
  int pose_is_obj_cam;            /* 1: t_cam_obj[] already holds t_obj_cam (teacher forcing) */
} dsr_object_in;

enum {
  DSR_OK = 0,
  DSR_FAIL_SDF_NAN = 1,           /* optimizer.py:137-138 */
  DSR_FAIL_RENDER_FEW = 2,        /* loss.py:86-88 -> optimizer.py:144-145 */
  DSR_FAIL_RENDER_NAN = 3         /* optimizer.py:151-152 (includes K == 0) */
};

typedef struct {
  float t_cam_obj[16];            /* optimized object->camera (valid iff is_good) */
  float code[DSR_CODE_LEN];       /* optimized code (valid iff is_good) */
  float loss;                     /* k1*render + k2*sdf of the last iteration, pre-update */
  int is_good;
  int fail_reason;                /* DSR_FAIL_* */
  int iters_done;                 /* completed GN updates */
  int n_valid_last, k_last;       /* ray samples in the unit ball / render points, last iter */
} dsr_object_out;

/* Optional per-iteration trace for tests (teacher-forced parity).  Arrays are
 * [num_iterations] (H: [num_iterations][71*71]) for ONE object; the caller
 * allocates. */
typedef struct {
  float* H;                       /* damped normal matrix that is inverted (optimizer.py:188) */
  float* b;                       /* right-hand side */
  float* dx;                      /* inv(H) b */
  float* loss;                    /* k1*render+k2*sdf */
  float* sdf_loss;
  float* render_loss;
  int* n_valid;
  int* k;
  float* t_obj_cam;               /* [num_iterations][16] state the iteration started from */
  float* z;                       /* [num_iterations][code_len] */
  /* ABI 11 (may be NULL): the iteration's work counts — ray samples decoded by the render passes
     (early ray termination: every sample in front of a ray's first certainly-full one, plus
     those its pass window held behind it) and samples re-decoded exactly after the lite pass */
  int* n_decoded;
  int* n_refined;
} dsr_trace;

typedef struct {
  double fwd_ms;                  /* summed device time of the ray-sample decoder kernel */
  double jac_ms;                  /* summed device time of the fwd+Jacobian kernel */
  double total_ms;                /* wall (device events) of the last run */
  int64_t fwd_points;             /* ray samples decoded (early ray termination skips the
                                     samples behind a ray's first sdf <= -cut_off) */
  int64_t jac_points;             /* sum of (N + K) */
  int fwd_launches, jac_launches; /* fwd: one per render pass per iteration */
  int64_t inball_points;          /* sum over iterations/objects of N_valid (in-ball samples) */
  int lite;                       /* 1: fwd_* is the one-product lite pass (DSR_LITE) and
                                     refine_* the exact split-fp16 re-decode of its band */
  int refine_launches;
  double refine_ms;
  int64_t refine_points;
  double lite_max_err;            /* max |lite - exact| over the re-decoded samples (band and
                                     audited), all objects */
  double lite_min_margin;         /* smallest classification margin the last run used */
  int64_t jac_surface_points;     /* of jac_points: surface points N (forward + backward) */
  int64_t jac_render_points;      /* of jac_points: render points K (backward only when
                                     keep_masks, else forward + backward) */
  int keep_masks;                 /* 1: render points reuse the exact pass's ReLU masks */
  int lite_audit_violations;      /* audited out-of-band samples whose exact class (full /
                                     band / empty) differed from the lite pass's */
  int lite_redo_objects;          /* objects that discarded an iteration for a violation and
                                     finished with exact decoding */
  int surface_in_exact;           /* 1: the exact pass ran the surface points' forward too and
                                     the Jacobian kernel only backward chains (kept masks) */
  int64_t audit_points;           /* out-of-band samples re-decoded exactly as an audit */
  int lite_broken_blocks;         /* staggered lite-pass workgroups whose bounded event wait
                                     expired in the last run (their samples all went to the
                                     exact pass: results stay exact, the cost rises); 0 expected */
  int test_hooks;                 /* 1: the batch was created with DSR_TEST_HOOKS=1, so the test
                                     hooks (DSR_LITE_PERTURB / _BREAK) and the lite-guard settings
                                     below (DSR_LITE_AUDIT / _SHELL / _AUDIT_LOG2 / _MARGIN / _FLOOR /
                                     _SAFETY) were read from the environment */
  /* ---- the lite pass's guard as this batch ran it (ABI 8) ---- */
  int lite_eligible;              /* the decoder passed its load-time lite qualification
                                     (dsr_decoder_info); 0: every batch decodes exactly */
  int audit;                      /* 1: audited out-of-band samples (lite_flag) */
  float audit_shell;              /* certain audit of |y| < th + (1 + shell) * margin */
  int audit_log2;                 /* plus a hashed 2^-audit_log2 share of all other samples */
  float lite_margin0;             /* first-iteration margin */
  float lite_floor;               /* later margins: max(floor, safety x largest observed error) */
  float lite_safety;
  int graph_captures;             /* hipGraph captures / replays over the batch's life */
  int graph_replays;
  /* ---- the kernels and launch structure this batch ran (ABI 10) ---- */
  int n_groups;                   /* object groups on concurrent streams (DSR_STREAMS or the default) */
  int graph_mode;                 /* 0 eager, 1 DSR_GRAPH=1 (re-runs replay a graph), 2 a
                                     DSR_BATCH_GRAPH capacity batch */
  int fwd_variant;                /* exact-pass kernel (12: split-fp16, the shipped kernel) */
  int jac_variant;                /* Jacobian kernel (12: split-fp16) */
  int lite_variant;               /* lite-pass kernel (1496 shipped; 0 when the lite pass is off) */
  int split_ring;                 /* A-ring depth of the split kernels (2 shipped).  Only under
                                     DSR_TEST_HOOKS=1 can DSR_FWD_VARIANT / _JAC_VARIANT /
                                     _LITE_VARIANT / _SPLIT_RING move these from the shipped values.
                                     ABI 11: the four are the kernels the last run DISPATCHED
                                     (recorded as it was enqueued), not the environment's values */
  int prescan;                    /* ABI 11: 1 if the render passes ran over the ray chunks
                                     (k_sample_scan / k_sample_count + k_sample_emit; one-group
                                     batches), 0 for one workgroup per object (k_sample_pass) */
} dsr_stats;

/* ---- context ------------------------------------------------------------- */
int dsr_abi_version(void);
int dsr_ctx_create(int device, dsr_ctx** out);
int dsr_ctx_destroy(dsr_ctx* ctx);
const char* dsr_last_error(const dsr_ctx* ctx);
int dsr_device_count(int* n);

/* ---- decoder: replaces deep_sdf.workspace.config_decoder (workspace.py:202-223)
 * + reconstruct.utils.get_decoder (utils.py:93-94).  `weights` holds the folded
 * (weight-norm applied, W = g*v/||v||) layers back to back: for each layer i,
 * W_i (out_dim x in_dim, row-major) then b_i (out_dim). */
int dsr_decoder_load(dsr_ctx* ctx, const dsr_decoder_desc* desc, const float* weights,
                     size_t n_floats, dsr_decoder** out);
int dsr_decoder_free(dsr_ctx* ctx, dsr_decoder* dec);

/* Load-time qualification of the one-product fp16 classification pass (no reference
 * counterpart; it guards the build's replacement of decode_sdf, loss_utils.py:51-79, in the
 * render term's occupancy classification, loss.py:98-102 / loss_utils.py:40-48).
 * dsr_decoder_load decodes a fixed probe set — probe_points points uniform in the unit ball x
 * probe_codes latent codes (zero, then N(0, s^2) per component for s = 0.1, 0.3, 1.0) — with
 * the lite pass and with the exact split-fp16 pass and records, over every probe value, the
 * largest |lite - exact| / max(floor, ||exact| - th|) (th = 0.01, floor = 0.002): the lite
 * error as a fraction of the distance of the exact value to the nearest class boundary
 * (full | band | empty), and the largest |lite - exact| near the surface (|exact| < 0.1).  A
 * decoder whose ratio exceeds 0.5, or whose near-surface error exceeds half the floor (1e-3), is
 * lite-ineligible: every batch on it decodes every ray sample exactly (the DSR_LITE=0 path,
 * reported in dsr_stats). */
typedef struct {
  int code_len;
  int lite_eligible;
  double lite_probe_ratio;        /* max |lite - exact| / max(floor, ||exact| - th|) */
  double lite_probe_max_err;      /* max |lite - exact| over probe values with |exact| < 0.1 */
  double lite_probe_max_err_all;  /* max |lite - exact| over every probe value */
  int probe_points, probe_codes;
  double probe_ms;                /* host wall time of the qualification */
} dsr_decoder_info;
int dsr_decoder_info_get(const dsr_decoder* dec, dsr_decoder_info* info);

/* ---- joint shape + pose GN: replaces Optimizer.reconstruct_object
 * (optimizer.py:90-205) for n_obj independent objects in one device pass.
 * `trace` may be NULL; if not, it must point to n_obj dsr_trace records. */
int dsr_reconstruct_batch(dsr_ctx* ctx, const dsr_decoder* dec, const dsr_optim_params* p,
                          int n_obj, const dsr_object_in* in, dsr_object_out* out,
                          const dsr_trace* trace);

/* Resident batches for benchmarking / streaming (inputs uploaded once; a run
 * re-initializes the optimizer state on device and executes all iterations on
 * the context stream). */
int dsr_batch_create(dsr_ctx* ctx, const dsr_decoder* dec, const dsr_optim_params* p,
                     int n_obj, const dsr_object_in* in, dsr_batch** out);
int dsr_batch_run(dsr_batch* b);                  /* async on the context stream; with
                                                      DSR_GRAPH=1 re-runs replay a hipGraph */
int dsr_batch_graph(dsr_batch* b);                /* capture that graph now (DSR_GRAPH=1) */
int dsr_batch_sync(dsr_batch* b);
int dsr_batch_query(dsr_batch* b);                /* 1: the last run has finished, 0: still in
                                                      flight (host work can overlap it), <0 error */
int dsr_batch_download(dsr_batch* b, dsr_object_out* out);
int dsr_batch_stats(dsr_batch* b, dsr_stats* st);
/* Diagnostics of the staggered lite pass (no reference counterpart): copies up to n ints of
 * the last run's record — [0] broken workgroups, [1] 1 if the first expired event wait was
 * recorded, then its workgroup, wave, counter, target, observed value, tile iteration,
 * HW_ID, XCC_ID, and how many polls took how many 100 MHz ticks before it expired
 * (csrc/dsr_dev.hpp: STD_*; 16 ints). */
int dsr_batch_lite_diag(dsr_batch* b, int* rec, int n);
int dsr_batch_destroy(dsr_batch* b);

/* Fixed-capacity batches for a keyframe stream (BASELINE config 5; the per-keyframe loop
 * LocalMapping_util.cc:256-445 / :165-206, overlapped with LocalMapping.cc:99-128): the batch
 * is laid out once for max_obj objects of at most max_pts surface points and max_rays rays,
 * and dsr_batch_refill uploads each keyframe's objects into those slots (host -> pinned
 * staging -> one stream-ordered copy per input buffer) and rewrites the per-slot counts in
 * device memory, so every kernel argument stays fixed.  With DSR_BATCH_GRAPH the whole GN run
 * is captured as ONE hipGraph at the first run and every later run — after any refill —
 * replays it (dsr_stats.graph_captures / graph_replays).  The batch starts empty; a run needs
 * a refill first; dsr_batch_download returns the current fill's n_obj records.  A refill
 * orders after the previous run's work on the context stream. */
#define DSR_BATCH_GRAPH 1
int dsr_batch_create_capacity(dsr_ctx* ctx, const dsr_decoder* dec, const dsr_optim_params* p, int max_obj,
                              int max_pts, int max_rays, int flags, dsr_batch** out);
int dsr_batch_refill(dsr_batch* b, int n_obj, const dsr_object_in* in);

/* ---- decoder queries: replaces decode_sdf / get_batch_sdf_jacobian
 * (loss_utils.py:51-113) as used by Optimizer.compute_sdf_loss_objectpoint_zhjd
 * (optimizer.py:207-213) and MeshExtractor.extract_mesh_from_code
 * (optimizer.py:224-233).  pts are decoder-frame xyz; jac (n x (code_len+3)) may
 * be NULL. */
int dsr_sdf_eval(dsr_ctx* ctx, const dsr_decoder* dec, const float* code, const float* pts,
                 int n, float* sdf, float* jac);

/* ---- mesh extraction: replaces MeshExtractor (optimizer.py:216-233) with
 * convert_sdf_voxels_to_mesh (utils.py:119-140).  `grid_pts` is the (vol_dim^3 x 3)
 * voxel grid of reconstruct.utils.create_voxel_grid (uploaded once, like the reference's
 * MeshExtractor.__init__); dsr_mesher_run decodes it with `code`, runs marching cubes
 * at `level` on device and copies out vertices (n_verts x 3, float) and faces
 * (n_faces x 3, int).  Worst-case capacities: 3*vol_dim^3 vertices and
 * 5*(vol_dim-1)^3 faces; on a smaller capacity the counts are still returned with
 * status -5 and nothing is copied. */
typedef struct dsr_mesher dsr_mesher;
int dsr_mesher_create(dsr_ctx* ctx, const dsr_decoder* dec, const float* grid_pts, int vol_dim,
                      dsr_mesher** out);
int dsr_mesher_run(dsr_mesher* m, const float* code, float level, float* verts, int vcap, int* faces,
                   int fcap, int* n_verts, int* n_faces);
int dsr_mesher_destroy(dsr_mesher* m);

/* ---- marching cubes on a caller's volume: replaces convert_sdf_voxels_to_mesh
 * (utils.py:119-140) called on its own.  `vol` is the (vol_dim, vol_dim, vol_dim) SDF
 * volume in C order (vol[(i*vol_dim + j)*vol_dim + k] at voxel (i, j, k), the order
 * MeshExtractor's grid decode produces it in); vertices come back as voxel index x 2/(vol_dim-1)
 * - 1 (the reference's spacing and origin shift), faces as vertex indices.  Same kernels,
 * capacities and -5 status as dsr_mesher_run; device scratch lives for the call only. */
int dsr_mc_volume(dsr_ctx* ctx, const float* vol, int vol_dim, float level, float* verts, int vcap,
                  int* faces, int fcap, int* n_verts, int* n_faces);

/* ---- multi-GPU from one process: replaces the per-detection loop
 * LocalMapping_util.cc:165-206 spread over devices.  ctx[g] / dec[g] are one context and
 * its decoder per device; objects are LPT-partitioned (cost n_rays*M + n_pts), each
 * device's shard runs on its own host thread, and ONE RCCL gather (ncclCommInitAll over the
 * devices, ncclGather of the fixed-size dsr_object_out records to ctx[0]'s device, ABI 11)
 * returns them; out[] is filled in input order (results bitwise equal to a one-device batch).
 * RCCL is loaded at run time; without it, or when it refuses the device list (two contexts
 * on one device), the records are gathered through host memory: *path (may be NULL) reports
 * DSR_GATHER_RCCL or DSR_GATHER_HOST.  One process per GPU is reconstruct/parallel.py. */
#define DSR_GATHER_HOST 0
#define DSR_GATHER_RCCL 1
int dsr_reconstruct_multi_ex(dsr_ctx* const* ctx, const dsr_decoder* const* dec, int n_dev,
                             const dsr_optim_params* p, int n_obj, const dsr_object_in* in,
                             dsr_object_out* out, int* path);
int dsr_reconstruct_multi(dsr_ctx* const* ctx, const dsr_decoder* const* dec, int n_dev,
                          const dsr_optim_params* p, int n_obj, const dsr_object_in* in,
                          dsr_object_out* out);   /* = _ex with path NULL */
/* Host-only (no device needed): the multi-device layout — dev[i] the device of object i (LPT),
 * slot[i] its record within that device's shard, *maxn the largest shard (every device's gather
 * slot holds maxn records; object i is record dev[i] * maxn + slot[i] of the gathered buffer). */
int dsr_gather_layout(int n_obj, const dsr_object_in* in, int num_depth_samples, int n_dev, int* dev,
                      int* slot, int* maxn);

/* ---- pose-only SE(3) GN: replaces Optimizer.estimate_pose_cam_obj
 * (optimizer.py:46-87).  t_co_se3: 4x4 SE(3) camera<-object, scale: object scale,
 * result written to t_out (4x4). */
int dsr_pose_only(dsr_ctx* ctx, const dsr_decoder* dec, const dsr_optim_params* p,
                  const float* t_co_se3, float scale, const float* pts, int n_pts,
                  const float* code, float* t_out);

/* Batched form for the stereo path's per-keyframe loop over associated objects
 * (LocalMapping_util.cc:103-110 calls estimate_pose_cam_obj once per object): every
 * object's pose-only GN in one device pass per iteration.  t_out: n_obj x 16. */
typedef struct {
  float t_co_se3[16];             /* SE(3) camera<-object */
  float scale;
  const float* pts;               /* (n_pts,3) camera frame */
  int n_pts;
  const float* code;              /* (code_len,) */
} dsr_pose_in;
int dsr_pose_only_batch(dsr_ctx* ctx, const dsr_decoder* dec, const dsr_optim_params* p,
                        int n_obj, const dsr_pose_in* in, float* t_out);

#ifdef __cplusplus
}
#endif
#endif /* DSR_H */

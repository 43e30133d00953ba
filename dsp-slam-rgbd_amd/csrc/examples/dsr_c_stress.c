/*
 * dsr_c_stress.c — every entry point of the C ABI (include/dsr.h) from C, for the host-side
 * sanitizer build (Makefile: dsr_c_stress_asan = this file + libdsr_asan.so, host code under
 * AddressSanitizer + UndefinedBehaviorSanitizer; device code is the normal gfx950 build).
 *
 *   dsr_c_stress               no-device paths: ABI version, argument validation and error
 *                              reporting of every entry point that checks its arguments before
 *                              touching the device, context creation (-3 without a device)
 *   dsr_c_stress <dir>         the same inputs as dsr_c_smoke (weights.f32, params.f32,
 *                              objects.bin), then every device entry point with cross-checks:
 *                              one-shot batch twice (bitwise), resident batch create / run /
 *                              query / download / stats / lite diag / destroy, pooled re-create,
 *                              graph capture + replays (DSR_GRAPH=1), multi-context
 *                              reconstruct_multi, sdf_eval with and without the Jacobian,
 *                              pose-only single and batched (including an empty object), the
 *                              mesher (and dsr_mc_volume on its decoded grid) with ample and
 *                              with too small capacities, forced audit
 *                              violations and their spare-iteration redo (test hooks), and the
 *                              error paths of a live context.  Exit status 0 = every check held.
 */
#define _POSIX_C_SOURCE 200112L   /* setenv / unsetenv */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include "dsr.h"

static int n_checks = 0;
#define CHECK(cond, ...)                                                     \
  do {                                                                       \
    ++n_checks;                                                              \
    if (!(cond)) {                                                           \
      fprintf(stderr, "check failed (%s:%d): %s: ", __FILE__, __LINE__, #cond); \
      fprintf(stderr, __VA_ARGS__);                                          \
      fprintf(stderr, "\n");                                                 \
      exit(20);                                                              \
    }                                                                        \
  } while (0)

static void* slurp(const char* dir, const char* name, size_t* bytes) {
  char path[4096];
  snprintf(path, sizeof path, "%s/%s", dir, name);
  FILE* f = fopen(path, "rb");
  if (!f) return NULL;
  fseek(f, 0, SEEK_END);
  *bytes = (size_t)ftell(f);
  fseek(f, 0, SEEK_SET);
  void* p = malloc(*bytes ? *bytes : 1);
  if (p && fread(p, 1, *bytes, f) != *bytes) { free(p); p = NULL; }
  fclose(f);
  return p;
}

/* DSR_STRESS_SKIP="graph,multi,...": leave sections out (to attribute a sanitizer report) */
static int run_section(const char* name) {
  const char* skip = getenv("DSR_STRESS_SKIP");
  return !(skip && strstr(skip, name));
}

static const dsr_decoder_desc DESC = {64, 9, {512, 512, 512, 445, 512, 512, 512, 512, 1},
                                      {67, 512, 512, 512, 512, 512, 512, 512, 512}, 4, 0, 0};

static int same_out(const dsr_object_out* a, const dsr_object_out* b, int n) {
  return memcmp(a, b, sizeof(dsr_object_out) * (size_t)n) == 0;
}

/* argument validation that needs no device (the CPU-container case) */
static void no_device_paths(void) {
  CHECK(dsr_abi_version() == DSR_ABI_VERSION, "ABI %d", dsr_abi_version());
  int n = -1;
  const int rc = dsr_device_count(&n);
  CHECK(rc == 0 || rc < 0, "device_count %d", rc);
  CHECK(dsr_device_count(NULL) < 0, "device_count(NULL) accepted");
  CHECK(dsr_ctx_create(0, NULL) < 0, "ctx_create(NULL) accepted");
  CHECK(dsr_last_error(NULL) != NULL, "last_error(NULL) is NULL");
  CHECK(dsr_ctx_destroy(NULL) == 0, "ctx_destroy(NULL)");
  CHECK(dsr_batch_destroy(NULL) == 0, "batch_destroy(NULL)");
  CHECK(dsr_batch_run(NULL) < 0 && dsr_batch_sync(NULL) < 0 && dsr_batch_query(NULL) < 0,
        "batch calls on NULL accepted");
  CHECK(dsr_batch_download(NULL, NULL) < 0 && dsr_batch_stats(NULL, NULL) < 0, "batch NULL accepted");
  CHECK(dsr_mesher_destroy(NULL) == 0, "mesher_destroy(NULL)");
  CHECK(dsr_batch_refill(NULL, 0, NULL) < 0, "refill(NULL) accepted");
  CHECK(dsr_batch_create_capacity(NULL, NULL, NULL, 1, 1, 1, 0, NULL) < 0, "create_capacity(NULL) accepted");
  CHECK(dsr_decoder_info_get(NULL, NULL) < 0, "decoder_info_get(NULL) accepted");
  {
    float v[8] = {0};
    int nv = 0, nf = 0;
    CHECK(dsr_mc_volume(NULL, v, 2, 0.f, NULL, 0, NULL, 0, &nv, &nf) < 0, "mc_volume(NULL ctx) accepted");
  }
  dsr_ctx* c = NULL;
  const int rc2 = dsr_ctx_create(-7, &c);
  CHECK(rc2 < 0 && c == NULL, "ctx_create(-7) = %d", rc2);
}

/* error paths of a live context: every one returns < 0 with a message, none crashes */
static void live_error_paths(dsr_ctx* ctx, const dsr_decoder* dec, const float* w, size_t nw,
                             const dsr_optim_params* p, const dsr_object_in* in) {
  dsr_decoder* d2 = NULL;
  dsr_decoder_desc bad = DESC;
  bad.use_tanh = 2;
  CHECK(dsr_decoder_load(ctx, &bad, w, nw, &d2) < 0 && d2 == NULL, "use_tanh 2 accepted");
  CHECK(strlen(dsr_last_error(ctx)) > 0, "no message");
  bad = DESC;
  bad.norm_mask = 0x100;                       /* a LayerNorm after lin8: not a DeepSDF layer */
  CHECK(dsr_decoder_load(ctx, &bad, w, nw, &d2) < 0 && d2 == NULL, "norm_mask 0x100 accepted");
  bad.norm_mask = 1;                           /* lin0's LayerNorm needs 2 x 512 more floats */
  CHECK(dsr_decoder_load(ctx, &bad, w, nw, &d2) < 0 && d2 == NULL, "short LayerNorm weights accepted");
  bad = DESC;
  bad.use_tanh = 1;                            /* a decoder variant: loads, never lite-eligible */
  CHECK(dsr_decoder_load(ctx, &bad, w, nw, &d2) == 0 && d2 != NULL, "use_tanh refused: %s", dsr_last_error(ctx));
  {
    dsr_decoder_info inf;
    CHECK(dsr_decoder_info_get(d2, &inf) == 0 && inf.lite_eligible == 0 && inf.code_len == 64, "use_tanh info");
  }
  CHECK(dsr_decoder_free(ctx, d2) == 0, "free");
  d2 = NULL;
  bad = DESC;
  bad.latent_in = 3;
  CHECK(dsr_decoder_load(ctx, &bad, w, nw, &d2) < 0, "latent_in 3 accepted");
  CHECK(dsr_decoder_load(ctx, &DESC, w, nw - 1, &d2) < 0, "short weights accepted");
  CHECK(dsr_decoder_load(ctx, &DESC, NULL, nw, &d2) < 0, "NULL weights accepted");
  dsr_optim_params q = *p;
  dsr_object_out out[1];
  q.code_len = 32;
  CHECK(dsr_reconstruct_batch(ctx, dec, &q, 1, in, out, NULL) < 0, "code_len mismatch accepted");
  q = *p;
  q.num_depth_samples = 65;
  CHECK(dsr_reconstruct_batch(ctx, dec, &q, 1, in, out, NULL) < 0, "M 65 accepted");
  q = *p;
  q.num_iterations = -1;
  CHECK(dsr_reconstruct_batch(ctx, dec, &q, 1, in, out, NULL) < 0, "iters -1 accepted");
  CHECK(dsr_reconstruct_batch(ctx, dec, p, 0, in, out, NULL) < 0, "n_obj 0 accepted");
  CHECK(dsr_reconstruct_batch(ctx, dec, p, 1, NULL, out, NULL) < 0, "NULL in accepted");
  dsr_batch* b = NULL;
  CHECK(dsr_batch_create(ctx, dec, p, 0, in, &b) < 0 && b == NULL, "empty batch accepted");
  /* more ray samples than 32-bit device offsets hold: refused before any input is read (the
     ray pointer below covers only the real object's rays) */
  dsr_object_in big = in[0];
  big.n_rays = 50000000;
  big.n_depth = 0;
  CHECK(dsr_batch_create(ctx, dec, p, 1, &big, &b) < 0 && b == NULL, "2.5e9-sample batch accepted");
  CHECK(strstr(dsr_last_error(ctx), "too large") != NULL, "%s", dsr_last_error(ctx));
  CHECK(dsr_sdf_eval(ctx, dec, NULL, NULL, 4, NULL, NULL) < 0, "sdf_eval NULLs accepted");
  dsr_mesher* m = NULL;
  CHECK(dsr_mesher_create(ctx, dec, NULL, 8, &m) < 0 && m == NULL, "mesher without grid accepted");
}

int main(int argc, char** argv) {
  setvbuf(stdout, NULL, _IOLBF, 0);   /* a sanitizer's exit-time report must not swallow it */
  no_device_paths();
  dsr_ctx* ctx = NULL;
  const int rc = dsr_ctx_create(0, &ctx);
  printf("dsr_ctx_create %d\n", rc);
  if (argc < 2) {
    if (ctx) dsr_ctx_destroy(ctx);
    CHECK(rc == 0 || rc == -3, "ctx_create %d", rc);
    printf("stress ok (no-device paths): %d checks\n", n_checks);
    return 0;
  }
  CHECK(rc == 0, "ctx_create %d: %s", rc, dsr_last_error(ctx));
  size_t wb = 0, pb = 0, ob = 0;
  float* w = (float*)slurp(argv[1], "weights.f32", &wb);
  float* pf = (float*)slurp(argv[1], "params.f32", &pb);
  char* objs = (char*)slurp(argv[1], "objects.bin", &ob);
  CHECK(w && pf && objs && pb >= 13 * sizeof(float), "missing inputs in %s", argv[1]);
  const size_t nw = wb / sizeof(float);
  dsr_decoder* dec = NULL;
  CHECK(dsr_decoder_load(ctx, &DESC, w, nw, &dec) == 0, "decoder_load: %s", dsr_last_error(ctx));
  const dsr_optim_params p = {pf[0], pf[1], pf[2], pf[3], pf[4], pf[5], pf[6], pf[7], (int)pf[8], (int)pf[9],
                              (int)pf[10], pf[11], (int)pf[12]};
  int n_obj = 0;
  memcpy(&n_obj, objs, sizeof(int));
  CHECK(n_obj > 0 && n_obj < 4096, "n_obj %d", n_obj);
  dsr_object_in* in = (dsr_object_in*)calloc((size_t)n_obj, sizeof(dsr_object_in));
  size_t off = sizeof(int);
  for (int o = 0; o < n_obj; ++o) {
    int hdr[3];
    memcpy(hdr, objs + off, sizeof hdr);
    off += sizeof hdr;
    memcpy(in[o].t_cam_obj, objs + off, 16 * sizeof(float));
    off += 16 * sizeof(float);
    in[o].pts = (const float*)(objs + off), in[o].n_pts = hdr[0];
    off += (size_t)3 * hdr[0] * sizeof(float);
    in[o].rays = (const float*)(objs + off), in[o].n_rays = hdr[1];
    off += (size_t)3 * hdr[1] * sizeof(float);
    in[o].depth = (const float*)(objs + off), in[o].n_depth = hdr[2];
    off += (size_t)hdr[2] * sizeof(float);
  }
  CHECK(off == ob, "objects.bin size mismatch");
  /* DSR_STRESS_MINIMAL=1: context + decoder + inputs only (what the runtime itself keeps) */
  const char* minimal = getenv("DSR_STRESS_MINIMAL");
  if (minimal && minimal[0] == '1') {
    CHECK(dsr_decoder_free(ctx, dec) == 0, "decoder_free");
    CHECK(dsr_ctx_destroy(ctx) == 0, "ctx_destroy");
    free(w); free(pf); free(objs); free(in);
    printf("stress ok (minimal): %d checks\n", n_checks);
    return 0;
  }
  const size_t osz = sizeof(dsr_object_out) * (size_t)n_obj;
  dsr_object_out* ref = (dsr_object_out*)calloc((size_t)n_obj, sizeof(dsr_object_out));
  dsr_object_out* out = (dsr_object_out*)calloc((size_t)n_obj, sizeof(dsr_object_out));

  /* one-shot batch, twice: deterministic */
  CHECK(dsr_reconstruct_batch(ctx, dec, &p, n_obj, in, ref, NULL) == 0, "%s", dsr_last_error(ctx));
  CHECK(dsr_reconstruct_batch(ctx, dec, &p, n_obj, in, out, NULL) == 0, "%s", dsr_last_error(ctx));
  CHECK(same_out(ref, out, n_obj), "one-shot batch not deterministic");
  int good = 0;
  for (int o = 0; o < n_obj; ++o) good += ref[o].is_good;
  CHECK(good > 0, "no object converged");

  /* per-object traces of the first object (caller-allocated arrays) */
  if (run_section("trace")) {
    const int it = p.num_iterations > 0 ? p.num_iterations : 1;
    dsr_trace* tr = (dsr_trace*)calloc((size_t)n_obj, sizeof(dsr_trace));
    float* H = (float*)calloc((size_t)it * 71 * 71, sizeof(float));
    float* b = (float*)calloc((size_t)it * 71, sizeof(float));
    float* dx = (float*)calloc((size_t)it * 71, sizeof(float));
    float* f3 = (float*)calloc((size_t)it * 3, sizeof(float));
    int* i2 = (int*)calloc((size_t)it * 2, sizeof(int));
    float* t = (float*)calloc((size_t)it * 16, sizeof(float));
    float* z = (float*)calloc((size_t)it * 64, sizeof(float));
    tr[0] = (dsr_trace){H, b, dx, f3, f3 + it, f3 + 2 * it, i2, i2 + it, t, z};
    CHECK(dsr_reconstruct_batch(ctx, dec, &p, n_obj, in, out, tr) == 0, "%s", dsr_last_error(ctx));
    CHECK(same_out(ref, out, n_obj), "traced batch differs");
    if (ref[0].iters_done > 0) CHECK(i2[0] > 0 && isfinite(H[0]), "empty trace");
    free(tr); free(H); free(b); free(dx); free(f3); free(i2); free(t); free(z);
  }

  /* resident batch: run / query / download / stats / diag, re-run, pooled re-create */
  for (int round = 0; round < 2 && run_section("resident"); ++round) {
    dsr_batch* bt = NULL;
    CHECK(dsr_batch_create(ctx, dec, &p, n_obj, in, &bt) == 0, "%s", dsr_last_error(ctx));
    for (int r = 0; r < 3; ++r) {
      memset(out, 0, osz);
      CHECK(dsr_batch_run(bt) == 0, "%s", dsr_last_error(ctx));
      int q, polls = 0;
      while ((q = dsr_batch_query(bt)) == 0) ++polls;
      CHECK(q == 1, "query %d", q);
      CHECK(dsr_batch_download(bt, out) == 0, "%s", dsr_last_error(ctx));
      CHECK(same_out(ref, out, n_obj), "resident run %d.%d differs (%d polls)", round, r, polls);
      dsr_stats st;
      CHECK(dsr_batch_stats(bt, &st) == 0, "%s", dsr_last_error(ctx));
      CHECK(st.fwd_points > 0 && st.lite_broken_blocks == 0 && st.test_hooks == 0, "stats");
      int rec[32];
      CHECK(dsr_batch_lite_diag(bt, rec, 32) >= 0, "%s", dsr_last_error(ctx));
      CHECK(rec[0] == 0, "broken blocks %d", rec[0]);
    }
    CHECK(dsr_batch_sync(bt) == 0, "%s", dsr_last_error(ctx));
    CHECK(dsr_batch_destroy(bt) == 0, "destroy");
  }

  /* audit violations forced through the test hooks (read at batch creation): every run
     discards iterations and redoes them in the spare iteration, enqueued by dsr_batch_query
     (first run) or by the download (second run) */
  if (run_section("redo")) {
    setenv("DSR_TEST_HOOKS", "1", 1);
    setenv("DSR_LITE_PERTURB", "0.015", 1);
    dsr_batch* bt = NULL;
    CHECK(dsr_batch_create(ctx, dec, &p, n_obj, in, &bt) == 0, "%s", dsr_last_error(ctx));
    unsetenv("DSR_TEST_HOOKS");
    unsetenv("DSR_LITE_PERTURB");
    for (int r = 0; r < 2; ++r) {
      memset(out, 0, osz);
      CHECK(dsr_batch_run(bt) == 0, "%s", dsr_last_error(ctx));
      int q = 0;
      if (r == 0)
        while ((q = dsr_batch_query(bt)) == 0) {}
      CHECK(q >= 0, "query %d", q);
      CHECK(dsr_batch_download(bt, out) == 0, "%s", dsr_last_error(ctx));
      dsr_stats st;
      CHECK(dsr_batch_stats(bt, &st) == 0, "%s", dsr_last_error(ctx));
      CHECK(st.test_hooks == 1 && st.lite_redo_objects > 0, "hooks %d redo %d", st.test_hooks, st.lite_redo_objects);
      for (int o = 0; o < n_obj; ++o)
        CHECK(!out[o].is_good || out[o].iters_done == p.num_iterations, "object %d: %d iterations", o,
              out[o].iters_done);
    }
    CHECK(dsr_batch_destroy(bt) == 0, "destroy");
  }

  /* fixed-capacity batch (keyframe stream): refilled fills, eager and as one replayed graph;
     the same objects in reverse slot order come back reversed, bitwise */
  if (run_section("capacity")) {
    dsr_decoder_info di;
    CHECK(dsr_decoder_info_get(dec, &di) == 0 && di.lite_eligible == 1 && di.probe_points == 65536,
          "decoder info: eligible %d ratio %g", di.lite_eligible, di.lite_probe_ratio);
    int mp = 0, mr = 0;
    for (int o = 0; o < n_obj; ++o) {
      mp = in[o].n_pts > mp ? in[o].n_pts : mp;
      mr = in[o].n_rays > mr ? in[o].n_rays : mr;
    }
    dsr_object_in* rev = (dsr_object_in*)calloc((size_t)n_obj, sizeof(dsr_object_in));
    for (int o = 0; o < n_obj; ++o) rev[o] = in[n_obj - 1 - o];
    /* (the graph-captured variant counts as part of the "graph" section: HIP keeps memory after
       a capture, which the differential leak test leaves out) */
    const int max_flags = run_section("graph") ? DSR_BATCH_GRAPH : 0;
    for (int flags = 0; flags <= max_flags; ++flags) {
      dsr_batch* bt = NULL;
      CHECK(dsr_batch_create_capacity(ctx, dec, &p, n_obj, mp, mr, flags, &bt) == 0, "%s", dsr_last_error(ctx));
      CHECK(dsr_batch_run(bt) < 0, "run of an empty capacity batch accepted");
      CHECK(dsr_batch_refill(bt, n_obj + 1, in) < 0, "refill beyond the object capacity accepted");
      for (int r = 0; r < 4; ++r) {
        const int back = r & 1;
        CHECK(dsr_batch_refill(bt, n_obj, back ? rev : in) == 0, "%s", dsr_last_error(ctx));
        memset(out, 0, osz);
        CHECK(dsr_batch_run(bt) == 0, "%s", dsr_last_error(ctx));
        CHECK(dsr_batch_download(bt, out) == 0, "%s", dsr_last_error(ctx));
        for (int o = 0; o < n_obj; ++o)
          CHECK(same_out(&ref[o], &out[back ? n_obj - 1 - o : o], 1), "capacity fill %d (flags %d) object %d", r,
                flags, o);
      }
      dsr_stats st;
      CHECK(dsr_batch_stats(bt, &st) == 0, "%s", dsr_last_error(ctx));
      CHECK(st.graph_captures == (flags ? 1 : 0) && st.graph_replays == (flags ? 4 : 0), "captures %d replays %d",
            st.graph_captures, st.graph_replays);
      CHECK(dsr_batch_destroy(bt) == 0, "destroy");
    }
    dsr_batch* bt = NULL;
    CHECK(dsr_batch_create(ctx, dec, &p, n_obj, in, &bt) == 0, "%s", dsr_last_error(ctx));
    CHECK(dsr_batch_refill(bt, n_obj, in) < 0, "refill of an ordinary batch accepted");
    CHECK(dsr_batch_destroy(bt) == 0, "destroy");
    free(rev);
  }

  /* graph capture and replays */
  setenv("DSR_GRAPH", "1", 1);
  if (run_section("graph")) {
    dsr_batch* bt = NULL;
    CHECK(dsr_batch_create(ctx, dec, &p, n_obj, in, &bt) == 0, "%s", dsr_last_error(ctx));
    CHECK(dsr_batch_graph(bt) == 0, "%s", dsr_last_error(ctx));
    for (int r = 0; r < 4; ++r) {
      memset(out, 0, osz);
      CHECK(dsr_batch_run(bt) == 0, "%s", dsr_last_error(ctx));
      CHECK(dsr_batch_download(bt, out) == 0, "%s", dsr_last_error(ctx));
      CHECK(same_out(ref, out, n_obj), "graph replay %d differs", r);
    }
    CHECK(dsr_batch_destroy(bt) == 0, "destroy");
  }
  unsetenv("DSR_GRAPH");

  /* two contexts on this device through the multi-device entry point */
  if (run_section("multi")) {
    dsr_ctx* c2 = NULL;
    dsr_decoder* d2 = NULL;
    CHECK(dsr_ctx_create(0, &c2) == 0, "second context");
    CHECK(dsr_decoder_load(c2, &DESC, w, nw, &d2) == 0, "%s", dsr_last_error(c2));
    dsr_ctx* cs[2] = {ctx, c2};
    const dsr_decoder* ds[2] = {dec, d2};
    memset(out, 0, osz);
    CHECK(dsr_reconstruct_multi(cs, ds, 2, &p, n_obj, in, out) == 0, "%s", dsr_last_error(ctx));
    CHECK(same_out(ref, out, n_obj), "reconstruct_multi differs");
    CHECK(dsr_decoder_free(c2, d2) == 0, "decoder_free");
    CHECK(dsr_ctx_destroy(c2) == 0, "ctx_destroy");
  }

  /* decoder queries: sdf with and without the Jacobian, at the first object's code */
  if (run_section("query")) {
    const int n = 1000;
    float* x = (float*)malloc(sizeof(float) * 3 * n);
    float* s0 = (float*)malloc(sizeof(float) * n);
    float* s1 = (float*)malloc(sizeof(float) * n);
    float* J = (float*)malloc(sizeof(float) * (size_t)n * 67);
    unsigned r = 12345u;
    for (int i = 0; i < 3 * n; ++i) {
      r = r * 1664525u + 1013904223u;
      x[i] = ((float)(r >> 8) / 16777216.f) * 1.8f - 0.9f;
    }
    CHECK(dsr_sdf_eval(ctx, dec, ref[0].code, x, n, s0, NULL) == 0, "%s", dsr_last_error(ctx));
    CHECK(dsr_sdf_eval(ctx, dec, ref[0].code, x, n, s1, J) == 0, "%s", dsr_last_error(ctx));
    for (int i = 0; i < n; ++i) CHECK(isfinite(s0[i]) && fabsf(s0[i] - s1[i]) <= 2e-6f, "sdf %d", i);
    for (int i = 0; i < n * 67; ++i) CHECK(isfinite(J[i]), "jac %d", i);
    CHECK(dsr_sdf_eval(ctx, dec, NULL, x, n, s0, NULL) < 0, "NULL code accepted");
    CHECK(dsr_sdf_eval(ctx, dec, ref[0].code, x, 0, NULL, NULL) == 0, "n = 0: %s", dsr_last_error(ctx));

    /* pose-only: single vs batch; an empty object gives NaN in its slot only */
    float T1[16], Tb[3 * 16];
    const float* z = ref[0].code;
    float Tse3[16];
    memcpy(Tse3, in[0].t_cam_obj, sizeof Tse3);
    float sc = cbrtf(Tse3[0] * (Tse3[5] * Tse3[10] - Tse3[6] * Tse3[9]) - Tse3[1] * (Tse3[4] * Tse3[10] - Tse3[6] * Tse3[8]) +
                     Tse3[2] * (Tse3[4] * Tse3[9] - Tse3[5] * Tse3[8]));
    for (int rr = 0; rr < 3; ++rr)
      for (int cc = 0; cc < 3; ++cc) Tse3[4 * rr + cc] /= sc;
    CHECK(dsr_pose_only(ctx, dec, &p, Tse3, sc, in[0].pts, in[0].n_pts, z, T1) == 0, "%s", dsr_last_error(ctx));
    dsr_pose_in pin[3];
    for (int k = 0; k < 3; ++k) {
      memcpy(pin[k].t_co_se3, Tse3, sizeof Tse3);
      pin[k].scale = sc;
      pin[k].pts = in[0].pts;
      pin[k].n_pts = k == 1 ? 0 : in[0].n_pts;
      pin[k].code = z;
    }
    CHECK(dsr_pose_only_batch(ctx, dec, &p, 3, pin, Tb) == 0, "%s", dsr_last_error(ctx));
    CHECK(memcmp(T1, Tb, sizeof T1) == 0 && memcmp(T1, Tb + 32, sizeof T1) == 0, "pose batch != single");
    CHECK(isnan(Tb[16]), "empty object not NaN");
    free(x); free(s0); free(s1); free(J);
  }

  /* mesher: a d^3 grid over [-1, 1]^3, ample capacities, then too small ones (-5, counts) */
  if (run_section("mesher")) {
    const int d = 24;
    const size_t nv = (size_t)d * d * d;
    float* grid = (float*)malloc(sizeof(float) * 3 * nv);
    for (int i = 0; i < d; ++i)
      for (int j = 0; j < d; ++j)
        for (int k = 0; k < d; ++k) {
          float* g = grid + 3 * (((size_t)i * d + j) * d + k);
          g[0] = -1.f + 2.f * i / (d - 1), g[1] = -1.f + 2.f * j / (d - 1), g[2] = -1.f + 2.f * k / (d - 1);
        }
    dsr_mesher* m = NULL;
    CHECK(dsr_mesher_create(ctx, dec, grid, d, &m) == 0, "%s", dsr_last_error(ctx));
    const int vcap = 3 * d * d * d, fcap = 5 * (d - 1) * (d - 1) * (d - 1);
    float* V = (float*)malloc(sizeof(float) * 3 * (size_t)vcap);
    int* F = (int*)malloc(sizeof(int) * 3 * (size_t)fcap);
    int nvert = -1, nface = -1, nv2 = -1, nf2 = -1;
    CHECK(dsr_mesher_run(m, ref[0].code, 0.f, V, vcap, F, fcap, &nvert, &nface) == 0, "%s", dsr_last_error(ctx));
    CHECK(nvert > 0 && nface > 0, "empty mesh");
    for (int f = 0; f < 3 * nface; ++f) CHECK(F[f] >= 0 && F[f] < nvert, "face index %d", F[f]);
    CHECK(dsr_mesher_run(m, ref[0].code, 0.f, V, 1, F, 1, &nv2, &nf2) == -5, "small capacity accepted");
    CHECK(nv2 == nvert && nf2 == nface, "counts on -5");
    CHECK(dsr_mesher_destroy(m) == 0, "mesher_destroy");
    /* the same grid decoded by dsr_sdf_eval, meshed by dsr_mc_volume: the mesher's mesh */
    float* vol = (float*)malloc(sizeof(float) * nv);
    float* V2 = (float*)malloc(sizeof(float) * 3 * (size_t)vcap);
    int* F2 = (int*)malloc(sizeof(int) * 3 * (size_t)fcap);
    CHECK(dsr_sdf_eval(ctx, dec, ref[0].code, grid, (int)nv, vol, NULL) == 0, "%s", dsr_last_error(ctx));
    nv2 = nf2 = -1;
    CHECK(dsr_mc_volume(ctx, vol, d, 0.f, V2, vcap, F2, fcap, &nv2, &nf2) == 0, "%s", dsr_last_error(ctx));
    CHECK(nv2 == nvert && nf2 == nface, "mc_volume counts %d/%d vs %d/%d", nv2, nf2, nvert, nface);
    CHECK(memcmp(V, V2, sizeof(float) * 3 * (size_t)nvert) == 0 && memcmp(F, F2, sizeof(int) * 3 * (size_t)nface) == 0,
          "mc_volume mesh differs from the mesher's");
    CHECK(dsr_mc_volume(ctx, vol, d, 0.f, V2, 1, F2, 1, &nv2, &nf2) == -5 && nv2 == nvert, "mc_volume small capacity");
    CHECK(dsr_mc_volume(ctx, NULL, d, 0.f, V2, vcap, F2, fcap, &nv2, &nf2) < 0, "mc_volume without volume");
    CHECK(dsr_mc_volume(ctx, vol, 1, 0.f, V2, vcap, F2, fcap, &nv2, &nf2) < 0, "mc_volume vol_dim 1 accepted");
    free(vol); free(V2); free(F2);
    free(grid); free(V); free(F);
  }

  if (run_section("errors")) live_error_paths(ctx, dec, w, nw, &p, in);
  /* the context still works after its errors */
  memset(out, 0, osz);
  CHECK(dsr_reconstruct_batch(ctx, dec, &p, n_obj, in, out, NULL) == 0, "%s", dsr_last_error(ctx));
  CHECK(same_out(ref, out, n_obj), "batch after error paths differs");

  CHECK(dsr_decoder_free(ctx, dec) == 0, "decoder_free");
  CHECK(dsr_ctx_destroy(ctx) == 0, "ctx_destroy");
  free(w); free(pf); free(objs); free(in); free(ref); free(out);
  printf("stress ok: %d checks, %d objects (%d good)\n", n_checks, n_obj, good);
  /* DSR_STRESS_QUICK_EXIT=1: skip the HIP runtime's static destructors (with host ASan, the
     sanitizer's device-allocator hook trips over the runtime freeing memory after its own
     teardown — at process exit, after every libdsr object here was destroyed) */
  const char* qe = getenv("DSR_STRESS_QUICK_EXIT");
  if (qe && qe[0] == '1') {
    fflush(stdout);
    _exit(0);
  }
  return 0;
}

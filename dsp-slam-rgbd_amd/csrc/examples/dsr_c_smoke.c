/*
 * dsr_c_smoke.c — the C ABI (include/dsr.h) from a C caller, without Python: what a C++
 * integration of libdsr under ORB-SLAM2 would do instead of the pybind11 route
 * (INTEGRATION.md §2).  Built by `make -C dsp-slam-rgbd_amd/csrc` next to libdsr.so.
 *
 *   dsr_c_smoke                 ABI version check + context creation only (prints the status;
 *                               -3 = no HIP device, the CPU-container case)
 *   dsr_c_smoke <dir>           loads <dir>/weights.f32 (folded lin0..lin8, W then b per layer),
 *                               <dir>/params.f32 (k1 k2 k3 k4 b1 b2 lr s_damp iters code_len M
 *                               cut_off pose_iters, all as float), <dir>/objects.bin (int32 n_obj,
 *                               then per object: int32 n_pts n_rays n_depth, float32 t_cam_obj[16],
 *                               pts[3 n_pts], rays[3 n_rays], depth[n_depth]), runs
 *                               dsr_reconstruct_batch and writes the dsr_object_out records to
 *                               <dir>/out.bin
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "dsr.h"

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

int main(int argc, char** argv) {
  if (dsr_abi_version() != DSR_ABI_VERSION) { fprintf(stderr, "ABI mismatch\n"); return 10; }
  dsr_ctx* ctx = NULL;
  const int rc = dsr_ctx_create(0, &ctx);
  printf("dsr_ctx_create %d\n", rc);
  if (argc < 2) { if (ctx) dsr_ctx_destroy(ctx); return (rc == 0 || rc == -3) ? 0 : 11; }
  if (rc) return 12;
  size_t wb = 0, pb = 0, ob = 0;
  float* w = (float*)slurp(argv[1], "weights.f32", &wb);
  float* pf = (float*)slurp(argv[1], "params.f32", &pb);
  char* objs = (char*)slurp(argv[1], "objects.bin", &ob);
  if (!w || !pf || !objs || pb < 13 * sizeof(float)) { fprintf(stderr, "missing inputs\n"); return 13; }
  const dsr_decoder_desc desc = {64, 9, {512, 512, 512, 445, 512, 512, 512, 512, 1},
                                 {67, 512, 512, 512, 512, 512, 512, 512, 512}, 4, 0, 0};
  dsr_decoder* dec = NULL;
  if (dsr_decoder_load(ctx, &desc, w, wb / sizeof(float), &dec)) { fprintf(stderr, "%s\n", dsr_last_error(ctx)); return 14; }
  dsr_optim_params p = {pf[0], pf[1], pf[2], pf[3], pf[4], pf[5], pf[6], pf[7], (int)pf[8], (int)pf[9],
                        (int)pf[10], pf[11], (int)pf[12]};
  int n_obj = 0;
  memcpy(&n_obj, objs, sizeof(int));
  dsr_object_in* in = (dsr_object_in*)calloc((size_t)n_obj, sizeof(dsr_object_in));
  dsr_object_out* out = (dsr_object_out*)calloc((size_t)n_obj, sizeof(dsr_object_out));
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
    in[o].code = NULL;
    in[o].pose_is_obj_cam = 0;
  }
  if (off != ob) { fprintf(stderr, "objects.bin size mismatch\n"); return 15; }
  if (dsr_reconstruct_batch(ctx, dec, &p, n_obj, in, out, NULL)) { fprintf(stderr, "%s\n", dsr_last_error(ctx)); return 16; }
  char path[4096];
  snprintf(path, sizeof path, "%s/out.bin", argv[1]);
  FILE* f = fopen(path, "wb");
  if (!f || fwrite(out, sizeof(dsr_object_out), (size_t)n_obj, f) != (size_t)n_obj) return 17;
  fclose(f);
  for (int o = 0; o < n_obj; ++o) printf("object %d: is_good %d loss %.6f iters %d\n", o, out[o].is_good, out[o].loss, out[o].iters_done);
  dsr_decoder_free(ctx, dec);
  dsr_ctx_destroy(ctx);
  free(w); free(pf); free(objs); free(in); free(out);
  return 0;
}

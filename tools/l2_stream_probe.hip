// L2 -> CU streaming rate probe (round 6): every wave of a 512-thread workgroup per CU streams
// 1 KiB fragments (16 B per lane, buffer loads, as the lite kernel's A ring does) from an
// L2-resident weight-sized buffer, NFRAG loads in flight per wave; prints GB/s and B/clk/CU.
// Answers whether a CU can take twice the lite kernel's weight stream.
// build: hipcc -O3 --offload-arch=gfx950 -o /tmp/l2_stream_probe tools/l2_stream_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef unsigned uint4v __attribute__((ext_vector_type(4)));

template <int NFRAG>
__global__ __launch_bounds__(512) void stream(const unsigned* __restrict__ buf, int frags, int iters,
                                              unsigned* __restrict__ out) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<unsigned*>(buf), 0,
                                                                     frags * 1024, 0x00020000);
  uint4v acc = {0u, 0u, 0u, 0u};
  int f = (blockIdx.x * 8 + w) * 7 % frags;
  for (int it = 0; it < iters; ++it) {
    uint4v v[NFRAG];
#pragma unroll
    for (int u = 0; u < NFRAG; ++u) {
      const int fi = (f + u * 13) % frags;
      v[u] = __builtin_bit_cast(uint4v, __builtin_amdgcn_raw_buffer_load_b128(r, lane * 16, fi * 1024, 0));
    }
#pragma unroll
    for (int u = 0; u < NFRAG; ++u) acc ^= v[u];
    f = (f + NFRAG * 13 + 1) % frags;
  }
  if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) out[blockIdx.x] = acc.x;   // keep the loads
}

int main() {
  int dev = 0, ncu = 0, clk_khz = 0;
  hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
  hipDeviceGetAttribute(&clk_khz, hipDeviceAttributeClockRate, dev);
  const int frags = 3584;                     // 3.5 MiB: the lite weight set's size, one XCD's L2
  unsigned* buf = nullptr;
  unsigned* out = nullptr;
  hipMalloc(&buf, (size_t)frags * 1024);
  hipMalloc(&out, sizeof(unsigned) * 4096);
  std::vector<unsigned> h((size_t)frags * 256);
  for (size_t i = 0; i < h.size(); ++i) h[i] = (unsigned)(i * 2654435761u);
  hipMemcpy(buf, h.data(), h.size() * 4, hipMemcpyHostToDevice);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const int iters = 2000;
  for (int pass = 0; pass < 2; ++pass) {
    auto run = [&](auto k, int nfrag, const char* name) {
      k<<<ncu, 512>>>(buf, frags, 10, out);
      hipDeviceSynchronize();
      hipEventRecord(a);
      k<<<ncu, 512>>>(buf, frags, iters, out);
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms = 0.f;
      hipEventElapsedTime(&ms, a, b);
      const double bytes = (double)ncu * 8 * iters * nfrag * 1024.0;
      const double gbs = bytes / (ms * 1e-3) / 1e9;
      const double bpc = bytes / ncu / (ms * 1e-3 * clk_khz * 1e3);
      if (pass) printf("%s: %.3f ms, %.0f GB/s, %.1f B/clk/CU (device clock %d MHz, %d CUs)\n", name, ms, gbs, bpc,
                       clk_khz / 1000, ncu);
    };
    run(stream<4>, 4, "4 loads in flight per wave");
    run(stream<8>, 8, "8 loads in flight per wave");
    run(stream<16>, 16, "16 loads in flight per wave");
  }
  hipFree(buf);
  hipFree(out);
  return 0;
}

// Stream-order probe (diagnostic; not product code).  Does a kernel launched after
// another on the SAME stream ever start while a workgroup of the earlier one is still running —
// the one mechanism that would explain §3.9's timing-dependent counts, which appear only while
// kernels of another hardware queue run beside?
//   producer<<<G, 64>>>: the LAST workgroup waits `delay` ticks of the 100 MHz clock, then stores
//                        the iteration's token; every other workgroup returns at once;
//   consumer<<<1, 64>>>: records the token it sees.
// Launched back to back on one stream, `iters` times; with `load` a second stream (its own
// hardware queue) keeps every CU busy with spin workgroups meanwhile.  A consumer that records a
// stale token started before its producer had finished.  All stores are vector stores.
#include <hip/hip_runtime.h>

__global__ void k_producer(int* flag, int token, long long delay) {
  if (blockIdx.x != gridDim.x - 1) return;
  if (threadIdx.x == 0) {
    const long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < delay) __builtin_amdgcn_s_sleep(8);
    __atomic_store_n(flag, token, __ATOMIC_RELEASE);
  }
}

__global__ void k_consumer(const int* flag, int* seen, int it) {
  if (threadIdx.x == 0) seen[it] = __atomic_load_n(flag, __ATOMIC_ACQUIRE);
}

__global__ void k_spin(float* sink, long long ticks) {
  const long long t0 = __builtin_amdgcn_s_memrealtime();
  float x = threadIdx.x;
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) x = x * 0.999f + 1.0f;
  if (x == -1.0f) sink[blockIdx.x] = x;    // never true: keeps the loop
}

// returns the number of stale tokens seen (consumer started early), -1 on a HIP error
extern "C" int stream_order_probe(int iters, int grid, long long delay, int load, long long spin_ticks,
                                  int spin_grid, int* stale_out) {
  int *flag, *seen;
  float* sink;
  hipStream_t s, s2;
  if (hipMalloc((void**)&flag, sizeof(int)) || hipMalloc((void**)&seen, sizeof(int) * iters) ||
      hipMalloc((void**)&sink, sizeof(float) * spin_grid) || hipStreamCreate(&s) || hipStreamCreate(&s2))
    return -1;
  (void)hipMemset(flag, 0, sizeof(int));
  (void)hipMemset(seen, 0, sizeof(int) * iters);
  (void)hipDeviceSynchronize();
  for (int it = 0; it < iters; ++it) {
    if (load && it % 16 == 0) k_spin<<<spin_grid, 256, 0, s2>>>(sink, spin_ticks);
    k_producer<<<grid, 64, 0, s>>>(flag, it + 1, delay);
    k_consumer<<<1, 64, 0, s>>>(flag, seen, it);
  }
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  int* h = new int[iters];
  (void)hipMemcpy(h, seen, sizeof(int) * iters, hipMemcpyDeviceToHost);
  int stale = 0;
  for (int it = 0; it < iters; ++it) stale += h[it] != it + 1;
  *stale_out = stale;
  delete[] h;
  (void)hipFree(flag);
  (void)hipFree(seen);
  (void)hipFree(sink);
  (void)hipStreamDestroy(s);
  (void)hipStreamDestroy(s2);
  return 0;
}

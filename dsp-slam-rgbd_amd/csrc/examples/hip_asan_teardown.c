/* The HIP runtime alone under host AddressSanitizer (no libdsr): create a device allocation,
 * free it, exit normally.  Whether ASan's device-allocator hook trips over the runtime's own
 * teardown at exit is then a property of the runtime, not of libdsr — the attribution behind
 * examples/dsr_c_stress.c's DSR_STRESS_QUICK_EXIT (VERDICT r3 "What's weak" 7). */
#include <stdio.h>
#include <hip/hip_runtime_api.h>

int main(void) {
  void* p = NULL;
  if (hipSetDevice(0) != hipSuccess) return 2;
  if (hipMalloc(&p, 1 << 20) != hipSuccess) return 3;
  if (hipMemset(p, 0, 1 << 20) != hipSuccess) return 4;
  if (hipDeviceSynchronize() != hipSuccess) return 5;
  if (hipFree(p) != hipSuccess) return 6;
  printf("hip teardown probe: allocation freed, exiting normally\n");
  fflush(stdout);
  return 0;
}

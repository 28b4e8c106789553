// host_register — cost of hipHostRegister on pageable buffers vs. the copy rate it would save
// (design input for the host-buffer path, nttmul.cpp run_host).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <chrono>

static double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main() {
  const size_t sizes[] = {64u << 20, 256u << 20, 1024u << 20};
  for (size_t bytes : sizes) {
    char *h = (char *)aligned_alloc(4096, bytes);
    memset(h, 1, bytes);  // first touch
    void *d;
    (void)hipMalloc(&d, bytes);
    double t0 = now();
    hipError_t e = hipHostRegister(h, bytes, hipHostRegisterDefault);
    double t1 = now();
    (void)hipMemcpy(d, h, bytes, hipMemcpyHostToDevice);
    double t2 = now();
    (void)hipMemcpy(d, h, bytes, hipMemcpyHostToDevice);
    double t3 = now();
    (void)hipHostUnregister(h);
    double t4 = now();
    (void)hipMemcpy(d, h, bytes, hipMemcpyHostToDevice);  // pageable
    double t5 = now();
    printf("%5zu MiB: register %.2f ms (%s)  H2D registered %.1f GB/s  unregister %.2f ms  "
           "H2D pageable %.1f GB/s\n",
           bytes >> 20, (t1 - t0) * 1e3, hipGetErrorString(e), bytes / (t3 - t2) / 1e9,
           (t4 - t3) * 1e3, bytes / (t5 - t4) / 1e9);
    (void)t2;
    (void)hipFree(d);
    free(h);
  }
  return 0;
}

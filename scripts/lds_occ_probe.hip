// Empirical workgroups-per-CU vs dynamic LDS size: each 256-thread workgroup spins ~20 us; a grid of
// 4 x CUs workgroups finishes in ~20 us x ceil(4 / resident-per-CU).
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void __launch_bounds__(256) spin(int* out, long long ticks) {
  extern __shared__ int lds[];
  lds[threadIdx.x] = threadIdx.x;
  __syncthreads();
  long long t0 = wall_clock64();
  while (wall_clock64() - t0 < ticks) {
  }
  if (threadIdx.x == 0) out[blockIdx.x] = lds[5];
}
int main() {
  int* out;
  (void)hipMalloc(&out, 1 << 20);
  int cus = 0;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  int rate = 0;
  (void)hipDeviceGetAttribute(&rate, hipDeviceAttributeWallClockRate, 0);  // kHz
  long long ticks = (long long)rate * 20 / 1000;                             // 20 us
  (void)hipFuncSetAttribute((const void*)spin, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  size_t sizes[] = {36 * 1024, 40 * 1024, 41 * 1024, 44 * 1024, 48 * 1024, 54112, 64 * 1024, 80 * 1024};
  for (size_t bytes : sizes)
  for (int per = 2; per <= 5; ++per) {
    for (int rep = 0; rep < 2; ++rep) {
      (void)hipEventRecord(a);
      hipLaunchKernelGGL(spin, dim3(cus * per), dim3(256), bytes, 0, out, ticks);
      (void)hipEventRecord(b);
      (void)hipEventSynchronize(b);
      float ms = 0;
      (void)hipEventElapsedTime(&ms, a, b);
      int occ = 0;
      (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, (const void*)spin, 256, bytes);
      if (rep) printf("per=%d lds=%6zu B  time=%7.1f us  (~%.2f rounds of 20us)  api_occ=%d\n", per, bytes, ms * 1e3, ms * 1e3 / 20.0, occ);
    }
  }
  return 0;
}

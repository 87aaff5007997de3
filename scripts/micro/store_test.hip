// Development microbenchmark (not part of the library): what does the PGD tile kernel's skeleton
// (2048 workgroups x 256 threads, 32x64 output tiles, float2 stores in the pass-B item order, LDS
// footprint, barriers) cost without any arithmetic or loads?
#include <hip/hip_runtime.h>
#include <stdint.h>

__global__ void __launch_bounds__(256) k_linear(float4* out, int64_t n4) {
  int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n4) out[i] = make_float4(1.f, 2.f, 3.f, 4.f);
}

template <bool LDS, bool SYNC>
__global__ void __launch_bounds__(256, 4) k_tile(float* out, int n0, int n1, int tiles1) {
  extern __shared__ float smem[];
  const int tile = blockIdx.x;
  const int ty0 = (tile / tiles1) * 32, tx0 = (tile % tiles1) * 64;
  const int it = threadIdx.x;
  const int a = (it & 3) + 4 * ((it >> 5) & 1);
  const int cb = ((it >> 2) & 7) + 8 * (it >> 6);
  float v = 1.0f;
  if (LDS) {
    smem[threadIdx.x] = (float)threadIdx.x;
    if (SYNC) __syncthreads();
    v = smem[(threadIdx.x + 1) & 255];
    if (SYNC) __syncthreads();
  }
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int gr = ty0 + 4 * a + u, gc = tx0 + 2 * cb;
    *reinterpret_cast<float2*>(out + (unsigned)(gr * n1 + gc)) = make_float2(v, v);
  }
}

// rows-major variant: each wave writes 2 full rows (64 lanes x float2 = 512 B per row-pair)
template <bool LDS>
__global__ void __launch_bounds__(256, 4) k_tile_rows(float* out, int n0, int n1, int tiles1) {
  extern __shared__ float smem[];
  const int tile = blockIdx.x;
  const int ty0 = (tile / tiles1) * 32, tx0 = (tile % tiles1) * 64;
  float v = 1.0f;
  if (LDS) {
    smem[threadIdx.x] = (float)threadIdx.x;
    __syncthreads();
    v = smem[(threadIdx.x + 1) & 255];
  }
  const int lane = threadIdx.x & 31, rw = threadIdx.x >> 5;  // 8 row slots of 32 lanes x float2
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int gr = ty0 + rw + 8 * u, gc = tx0 + 2 * lane;
    *reinterpret_cast<float2*>(out + (unsigned)(gr * n1 + gc)) = make_float2(v, v);
  }
}

extern "C" int run(int which, float* out, int n, int smem, hipStream_t s) {
  const int tiles1 = n / 64, tiles = (n / 32) * tiles1;
  switch (which) {
    case 0: hipLaunchKernelGGL(k_linear, dim3((unsigned)((int64_t)n * n / 4 / 256)), dim3(256), 0, s, (float4*)out, (int64_t)n * n / 4); break;
    case 1: hipLaunchKernelGGL((k_tile<false, false>), dim3(tiles), dim3(256), 0, s, out, n, n, tiles1); break;
    case 2: hipFuncSetAttribute((const void*)k_tile<true, false>, hipFuncAttributeMaxDynamicSharedMemorySize, smem);
            hipLaunchKernelGGL((k_tile<true, false>), dim3(tiles), dim3(256), smem, s, out, n, n, tiles1); break;
    case 3: hipFuncSetAttribute((const void*)k_tile<true, true>, hipFuncAttributeMaxDynamicSharedMemorySize, smem);
            hipLaunchKernelGGL((k_tile<true, true>), dim3(tiles), dim3(256), smem, s, out, n, n, tiles1); break;
    case 4: hipLaunchKernelGGL((k_tile_rows<false>), dim3(tiles), dim3(256), 0, s, out, n, n, tiles1); break;
    case 5: hipFuncSetAttribute((const void*)k_tile_rows<true>, hipFuncAttributeMaxDynamicSharedMemorySize, smem);
            hipLaunchKernelGGL((k_tile_rows<true>), dim3(tiles), dim3(256), smem, s, out, n, n, tiles1); break;
  }
  return (int)hipGetLastError();
}

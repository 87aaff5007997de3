// Occupancy probe for the fused PGD kernel (run on the GPU box): prints device LDS/VGPR limits and
// hipOccupancyMaxActiveBlocksPerMultiprocessor for each fp32 radius.
#include "../pyxu_amd/csrc/pgd_tv2d.hip"
#include <cstdio>
template <int R>
void probe() {
  using L = pxa::Layout<float, R>;
  auto k = pxa::pgd_tv2d_kernel<float, R, true, 1>;
  (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)L::BYTES);
  int nb = -1;
  hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, (const void*)k, pxa::kThreads, L::BYTES);
  hipFuncAttributes fa;
  (void)hipFuncGetAttributes(&fa, (const void*)k);
  printf("R=%d lds=%zu blocks/CU=%d (err %d) regs=%d maxthreads=%d\n", R, (size_t)L::BYTES, nb, (int)e, fa.numRegs,
         fa.maxThreadsPerBlock);
}
int main() {
  hipDeviceProp_t p;
  (void)hipGetDeviceProperties(&p, 0);
  printf("%s CUs=%d lds/block=%zu lds/CU=%zu maxShmOptin=%zu regs/CU=%d\n", p.gcnArchName, p.multiProcessorCount,
         p.sharedMemPerBlock, p.maxSharedMemoryPerMultiProcessor, p.sharedMemPerBlockOptin, p.regsPerMultiprocessor);
  probe<1>();
  probe<2>();
  probe<4>();
  probe<6>();
  probe<8>();
  return 0;
}

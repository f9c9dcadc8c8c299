// Experiment: theoretical occupancy (blocks per CU) of the row kernels, from the runtime's
// occupancy calculator.  Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I qmf_amd/csrc
#include "../../qmf_amd/csrc/wals.hip"

#include <cstdio>

template <typename K>
static void report(const char* name, K kernel, int threads) {
  int blocks = 0;
  hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, kernel, threads, 0);
  hipFuncAttributes at{};
  (void)hipFuncGetAttributes(&at, reinterpret_cast<const void*>(kernel));
  std::printf("%-36s blocks/CU %3d (%s)  regs %d  lds %zu  local %zu\n", name, blocks,
              hipGetErrorString(e), at.numRegs, at.sharedSizeBytes, at.localSizeBytes);
}

int main() {
  using namespace qmfx;
  report("wals_direct_kernel<float,8>", wals_direct_kernel<float, 8>, 64);
  report("wals_direct_kernel<float,4>", wals_direct_kernel<float, 4>, 64);
  report("wals_woodbury_kernel<float,8,4>", wals_woodbury_kernel<float, 8, 4>, 64);
  report("wals_woodbury_kernel<float,8,3>", wals_woodbury_kernel<float, 8, 3>, 64);
  report("wals_woodbury_kernel<float,8,2>", wals_woodbury_kernel<float, 8, 2>, 64);
  report("wals_woodbury_kernel<float,4,2>", wals_woodbury_kernel<float, 4, 2>, 64);
  return 0;
}

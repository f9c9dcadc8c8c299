// Row solves of the direct kernel (csrc/direct.h), fp32 instantiations: one translation
// unit per precision so the two compile in parallel.
#include "direct.h"

namespace qmfx {

#ifndef QMFX_KERNELS_ONLY
hipError_t launch_wals_direct(const SolveArgs<float>& a, int nt, hipStream_t s) {
  if (a.seg_mode != 0) return launch_wals_heavy(a, nt, s);  // wals_heavy.hip
#define CALL(N) launch_direct_mode<float, N, 0>(a, s)
  QMFX_NT_SWITCH(nt, CALL)
#undef CALL
}
#endif  // QMFX_KERNELS_ONLY

}  // namespace qmfx

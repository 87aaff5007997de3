// Kernel D instantiations (float); see pds_march.hpp.
#include "pds_march.hpp"

namespace pxa {
namespace pds {

PXA_PDS_RUN_D(float) {
#define PXA_D(P, I, U) dispatch_d<float, P, I, U>(R0, pd, np, M, nseg, w, z, src, zo, ao, q, st)
  if (!dual) return pd3o ? PXA_D(true, false, false) : PXA_D(false, false, false);
  if (pd3o) return iso ? PXA_D(true, true, true) : PXA_D(true, false, true);
  return iso ? PXA_D(false, true, true) : PXA_D(false, false, true);
#undef PXA_D
}

}  // namespace pds
}  // namespace pxa

// Kernel B instantiations (float); see pds3d.hpp.
#include "pds3d.hpp"

namespace pxa {
namespace pds {

int run_b(const PdsB<float>& pb, bool pd3o, int R, const PdsPtrs& P, hipStream_t st) {
  return pd3o ? dispatch_b<float, true>(R, pb, P, st) : dispatch_b<float, false>(R, pb, P, st);
}

}  // namespace pds
}  // namespace pxa

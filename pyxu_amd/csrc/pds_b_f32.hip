// Kernel B instantiations (float); see pds3d.hpp.
#include "pds3d.hpp"

namespace pxa {
namespace pds {

int run_b(const PdsB<float>& pb, int mode, int R, const PdsPtrs& P, hipStream_t st) {
  switch (mode) {
    case 0: return dispatch_b<float, 0>(R, pb, P, st);
    case 1: return dispatch_b<float, 1>(R, pb, P, st);
    default: return dispatch_b<float, 2>(R, pb, P, st);
  }
}

}  // namespace pds
}  // namespace pxa

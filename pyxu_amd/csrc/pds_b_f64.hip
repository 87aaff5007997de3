// Kernel B instantiations (double); see pds3d.hpp.
#include "pds3d.hpp"

namespace pxa {
namespace pds {

int run_b(const PdsB<double>& pb, int mode, int R, const PdsPtrs& P, hipStream_t st) {
  switch (mode) {
    case 0: return dispatch_b<double, 0>(R, pb, P, st);
    case 1: return dispatch_b<double, 1>(R, pb, P, st);
    default: return dispatch_b<double, 2>(R, pb, P, st);
  }
}

}  // namespace pds
}  // namespace pxa

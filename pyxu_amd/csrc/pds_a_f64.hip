// Kernel A instantiations (double); see pds3d.hpp.
#include "pds3d.hpp"

namespace pxa {
namespace pds {

int run_a(const PdsA<double>& pa, bool pd3o, int R0, int np, int64_t M, int nseg, const void* src, const void* z,
          void* xo, void* q, hipStream_t st) {
  return pd3o ? dispatch_a<double, true>(R0, pa, np, M, nseg, src, z, xo, q, st)
              : dispatch_a<double, false>(R0, pa, np, M, nseg, src, z, xo, q, st);
}

}  // namespace pds
}  // namespace pxa

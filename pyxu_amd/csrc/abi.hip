// Library information entry points.
#include "common.hpp"

extern "C" {

const char* pxa_version(void) { return "pyxu_amd 0.1.0 (gfx950)"; }

int pxa_abi_version(void) { return 1; }

const char* pxa_error_string(int code) {
  switch (code) {
    case PXA_OK:
      return "success";
    case PXA_ERR_ARG:
      return "pyxu_amd: invalid argument";
    case PXA_ERR_DTYPE:
      return "pyxu_amd: unsupported dtype";
    case PXA_ERR_UNSUPPORTED:
      return "pyxu_amd: request outside the supported envelope";
    default:
      return code > 0 ? hipGetErrorString((hipError_t)code) : "pyxu_amd: unknown error";
  }
}

// Process-wide kernel-selection knobs (A/B measurements and parity tests of kernel variants).
static int g_tuning[PXA_TUNE_COUNT] = {0};

int pxa_tuning(int key, int value) {
  if (key < 0 || key >= PXA_TUNE_COUNT) return PXA_ERR_ARG;
  const int prev = g_tuning[key];
  if (value >= 0) g_tuning[key] = value;
  return prev;
}

}  // extern "C"

namespace pxa {
int tuning(int key) { return (key >= 0 && key < PXA_TUNE_COUNT) ? g_tuning[key] : 0; }
}  // namespace pxa

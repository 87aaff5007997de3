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

#include <map>
#include <mutex>
#include <tuple>

namespace pxa {
int tuning(int key) { return (key >= 0 && key < PXA_TUNE_COUNT) ? g_tuning[key] : 0; }

int resident_grid(const void* kernel, int threads, size_t lds) {
  static std::mutex mu;
  static std::map<std::tuple<const void*, int, int, size_t>, int> cache;
  int dev = 0;
  (void)hipGetDevice(&dev);
  const auto key = std::make_tuple(kernel, dev, threads, lds);
  std::lock_guard<std::mutex> lock(mu);
  auto it = cache.find(key);
  if (it != cache.end()) return it->second;
  int cus = 0, per = 0;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kernel, threads, lds);
  int g = cus * (per > 0 ? per : 1) / 8 * 8;
  if (g < 8) g = 8;
  cache[key] = g;
  return g;
}
}  // namespace pxa

// Host-side internals shared by the libclipmi translation units.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <mutex>
#include <set>
#include <string>
#include <utility>
#include "../../include/clipmi.h"

int clipmi_fail(hipError_t e, const char* file, int line);
int clipmi_invalid(const std::string& msg);
void clipmi_set_error(const std::string& msg);

#define CLIPMI_REQUIRE(cond, msg) do { if (!(cond)) return clipmi_invalid(std::string(__func__) + ": " + (msg)); } while (0)
#define CLIPMI_HIP(call) do { hipError_t e_ = (call); if (e_ != hipSuccess) return clipmi_fail(e_, __FILE__, __LINE__); } while (0)
// Dynamic-LDS opt-in (hipFuncSetAttribute MaxDynamicSharedMemorySize) once per (kernel, device),
// thread-safe; recorded only when it succeeds.
inline hipError_t lds_optin(const void* fn, int bytes) {
  static std::mutex mu;
  static std::set<std::pair<const void*, int>> done;
  int dev = 0;
  (void)hipGetDevice(&dev);
  std::lock_guard<std::mutex> g(mu);
  const auto key = std::make_pair(fn, dev);
  if (done.count(key)) return hipSuccess;
  const hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
  if (e == hipSuccess) done.insert(key);
  return e;
}

#define CLIPMI_TRY(call) do { int s_ = (call); if (s_ != CLIPMI_OK) return s_; } while (0)


// ---- live kernel profiler (clipmi_prof_*): while armed for a variant label, launches with
// that label are bracketed by hipEvents on their own stream, so a caller can time one kernel
// family inside a real step without host synchronisation.
struct ProfScope {
  hipStream_t s;
  int slot;
  ProfScope(hipStream_t stream, const char* label, double flops);
  void finish(const char* label, double flops);
};

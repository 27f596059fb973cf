// Host-side internals shared by the libclipmi translation units.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <map>
#include <mutex>
#include <string>
#include <utility>
#include "../../include/clipmi.h"

int clipmi_fail(hipError_t e, const char* file, int line);
int clipmi_invalid(const std::string& msg);
void clipmi_set_error(const std::string& msg);

#define CLIPMI_REQUIRE(cond, msg) do { if (!(cond)) return clipmi_invalid(std::string(__func__) + ": " + (msg)); } while (0)
#define CLIPMI_HIP(call) do { hipError_t e_ = (call); if (e_ != hipSuccess) return clipmi_fail(e_, __FILE__, __LINE__); } while (0)
// Dynamic-LDS opt-in (hipFuncSetAttribute MaxDynamicSharedMemorySize) per (kernel, device), thread-safe:
// the attribute is raised whenever a launch asks for more bytes than any earlier one did (a kernel whose
// dynamic LDS scales with its arguments, e.g. ln_bwd_any_kernel's 32 * D bytes, may first run small);
// the largest successfully set size is recorded.
inline hipError_t lds_optin(const void* fn, int bytes) {
  static std::mutex mu;
  static std::map<std::pair<const void*, int>, int> done;
  int dev = 0;
  (void)hipGetDevice(&dev);
  std::lock_guard<std::mutex> g(mu);
  const auto key = std::make_pair(fn, dev);
  const auto it = done.find(key);
  if (it != done.end() && it->second >= bytes) return hipSuccess;
  const hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
  if (e == hipSuccess) done[key] = bytes;
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

// ---- deferred deterministic reductions (engine backward, bf16 path).  The second stage of a split-K
// weight gradient (fp32 slabs -> C, per-split bias partials -> bias_grad) or of a LayerNorm affine
// gradient (per-block partial rows -> dgamma / dbeta) is recorded instead of launched and executed by the
// workgroups of the next persistent 4-wave GEMM launch on the same stream, before their first item
// (gemm4.hip hosted_reduce): no launch of its own, so no reduce waits for CUs behind the other tower's
// persistent GEMMs.  Same arithmetic, same order as the standalone kernels (bitwise equal).
struct DeferredReduce {
  int kind;  // 0 none, 1 split-K slabs, 2 column partials
  // kind 1: C[m][n] = (beta ? C[m][n] : 0) + alpha * sum_z ws[z][m][n] (N % 4 == 0, 16-B aligned);
  //         bias_grad[m] += sum_z bws[z][m] when bws
  const float* ws; float* C; int64_t ldc; int M, N, splits; float alpha; int beta;
  const float* bws; float* bias_grad;
  // kind 2: column c < Dt of sum_p part[p * stride + c] -> out[c] (c < D) / out2[c - D] (+= when pbeta);
  //         Dt = out2 ? 2D : D, D % 4 == 0
  const float* part; int64_t stride; int P, D; float* out; float* out2; int pbeta;
};
// The calling thread's deferral slot (nullptr: reductions launch as usual).  An empty slot (kind 0) takes
// the next split-K / LayerNorm second stage; a persistent 4-wave bf16 GEMM launch executes a recorded one
// and empties the slot.
DeferredReduce*& deferred_slot();
// launch a recorded reduction on its own (the standalone kernels) and empty it
int launch_deferred(hipStream_t s, DeferredReduce& r);
int launch_partials_reduce(hipStream_t s, const DeferredReduce& r);  // kind 2 (norm.hip)
// column sums from P partial rows [P][N] (+= when beta), deterministic; fold: 64 x N floats (gemm.hip)
int colsum_partials_finish(hipStream_t s, const float* part, int P, int N, float* colsum, int beta, float* fold);
int64_t colsum_partials_ws(int P, int N);  // bytes for the partial rows (256-B aligned) + fold
// the adapter's fused forward (adapter_fused.hip): whether it covers a call, and the kernel
bool adapter_fused_ok(int dtype, int ln, int D, int A, int64_t ldx, int64_t ldy);
int adapter_fwd_fused(void* stream, int R, int D, int A, const void* x, int64_t ldx, const void* w_down,
                      const void* b_down, const void* w_up, const void* b_up, const void* ln_w, const void* ln_b,
                      float eps, void* y, int64_t ldy, void* pre, void* act, void* z, float* mean, float* rstd);

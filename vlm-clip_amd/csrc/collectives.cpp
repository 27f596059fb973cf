// Data-parallel exchanges of the contrastive step as C-ABI entry points over RCCL (SURVEY.md §8b:
// clipmi_allgather_embed / clipmi_reducescatter_grad / clipmi_allreduce_grads), for FFI hosts that run
// one process per GPU without torch.distributed.  The PyTorch host issues the same exchanges through
// torch.distributed (clipmi/towers.py ContrastiveFn, clipmi/trainer.py GradBucketReducer).
//   all-gather      the L2-normalised [B, E] features of every rank before the similarity GEMMs
//                   (the reference computes the [B, B] logits on one device, model_m.py:146-171)
//   reduce-scatter  the column-direction feature gradients back to their owners
//   all-reduce      the fp32 gradient arena (or a bucket of it): trainer.py:92's loss.backward summed
//                   over the data-parallel replicas
// RCCL (/opt/rocm/lib/librccl.so.1) is opened on first use with RTLD_LOCAL, so the library has no link-time
// dependency on it and never binds to another RCCL a host process may have loaded (PyTorch bundles its own).
#include <dlfcn.h>
#include <cstring>
#include <mutex>
#include "internal.h"

namespace {

constexpr int kIdBytes = 128;  // NCCL_UNIQUE_ID_BYTES
struct UniqueId {
  char internal[kIdBytes];
};
typedef void* Comm;
typedef int (*GetUniqueIdFn)(UniqueId*);
typedef int (*CommInitRankFn)(Comm*, int, UniqueId, int);
typedef int (*CommDestroyFn)(Comm);
typedef int (*AllGatherFn)(const void*, void*, size_t, int, Comm, hipStream_t);
typedef int (*ReduceScatterFn)(const void*, void*, size_t, int, int, Comm, hipStream_t);
typedef int (*AllReduceFn)(const void*, void*, size_t, int, int, Comm, hipStream_t);
typedef const char* (*ErrStrFn)(int);
// rccl.h enums: ncclFloat32 = 7, ncclBfloat16 = 9, ncclSum = 0
constexpr int kF32 = 7, kBF16 = 9, kSum = 0;

struct Rccl {
  bool ok = false;
  std::string why;
  GetUniqueIdFn get_unique_id = nullptr;
  CommInitRankFn comm_init_rank = nullptr;
  CommDestroyFn comm_destroy = nullptr;
  AllGatherFn all_gather = nullptr;
  ReduceScatterFn reduce_scatter = nullptr;
  AllReduceFn all_reduce = nullptr;
  ErrStrFn err_str = nullptr;
};

const Rccl& rccl() {
  static Rccl r;
  static std::once_flag once;
  std::call_once(once, [] {
    const char* names[] = {"librccl.so.1", "/opt/rocm/lib/librccl.so.1", "librccl.so"};
    void* h = nullptr;
    for (const char* n : names)
      if ((h = dlopen(n, RTLD_NOW | RTLD_LOCAL))) break;
    if (!h) {
      r.why = std::string("cannot open librccl: ") + dlerror();
      return;
    }
    r.get_unique_id = (GetUniqueIdFn)dlsym(h, "ncclGetUniqueId");
    r.comm_init_rank = (CommInitRankFn)dlsym(h, "ncclCommInitRank");
    r.comm_destroy = (CommDestroyFn)dlsym(h, "ncclCommDestroy");
    r.all_gather = (AllGatherFn)dlsym(h, "ncclAllGather");
    r.reduce_scatter = (ReduceScatterFn)dlsym(h, "ncclReduceScatter");
    r.all_reduce = (AllReduceFn)dlsym(h, "ncclAllReduce");
    r.err_str = (ErrStrFn)dlsym(h, "ncclGetErrorString");
    r.ok = r.get_unique_id && r.comm_init_rank && r.comm_destroy && r.all_gather && r.reduce_scatter &&
           r.all_reduce && r.err_str;
    if (!r.ok) r.why = "librccl lacks an expected symbol";
  });
  return r;
}

int rccl_fail(const Rccl& r, int code, const char* what) {
  clipmi_set_error(std::string(what) + ": RCCL error " + std::to_string(code) + " (" + r.err_str(code) + ")");
  return CLIPMI_ERR_HIP;
}

int dtype_code(int dtype) { return dtype == CLIPMI_BF16 ? kBF16 : kF32; }

}  // namespace

#define CLIPMI_RCCL(r) \
  do {                 \
    if (!(r).ok) {     \
      clipmi_set_error((r).why); \
      return CLIPMI_ERR_UNSUPPORTED; \
    }                  \
  } while (0)

extern "C" int clipmi_comm_unique_id(void* id) {
  CLIPMI_REQUIRE(id, "comm_unique_id: id buffer (128 bytes)");
  const Rccl& r = rccl();
  CLIPMI_RCCL(r);
  UniqueId u;
  const int e = r.get_unique_id(&u);
  if (e) return rccl_fail(r, e, "ncclGetUniqueId");
  memcpy(id, u.internal, kIdBytes);
  return CLIPMI_OK;
}

extern "C" int clipmi_comm_init(void** comm, const void* id, int nranks, int rank) {
  CLIPMI_REQUIRE(comm && id, "comm_init: comm / id");
  CLIPMI_REQUIRE(nranks >= 1 && rank >= 0 && rank < nranks, "comm_init: 0 <= rank < nranks");
  const Rccl& r = rccl();
  CLIPMI_RCCL(r);
  UniqueId u;
  memcpy(u.internal, id, kIdBytes);
  Comm c = nullptr;
  const int e = r.comm_init_rank(&c, nranks, u, rank);
  if (e) return rccl_fail(r, e, "ncclCommInitRank");
  *comm = c;
  return CLIPMI_OK;
}

extern "C" int clipmi_comm_destroy(void* comm) {
  if (!comm) return CLIPMI_OK;
  const Rccl& r = rccl();
  CLIPMI_RCCL(r);
  const int e = r.comm_destroy((Comm)comm);
  if (e) return rccl_fail(r, e, "ncclCommDestroy");
  return CLIPMI_OK;
}

extern "C" int clipmi_allgather_embed(void* stream, void* comm, int dtype, const void* local, void* global,
                                      int64_t count) {
  CLIPMI_REQUIRE(comm && count >= 0 && (dtype == CLIPMI_F32 || dtype == CLIPMI_BF16), "allgather_embed: args");
  if (count == 0) return CLIPMI_OK;
  CLIPMI_REQUIRE(local && global, "allgather_embed: buffers");
  const Rccl& r = rccl();
  CLIPMI_RCCL(r);
  const int e = r.all_gather(local, global, (size_t)count, dtype_code(dtype), (Comm)comm, (hipStream_t)stream);
  if (e) return rccl_fail(r, e, "ncclAllGather");
  return CLIPMI_OK;
}

extern "C" int clipmi_reducescatter_grad(void* stream, void* comm, int dtype, const void* global, void* local,
                                         int64_t count) {
  CLIPMI_REQUIRE(comm && count >= 0 && (dtype == CLIPMI_F32 || dtype == CLIPMI_BF16), "reducescatter_grad: args");
  if (count == 0) return CLIPMI_OK;
  CLIPMI_REQUIRE(local && global, "reducescatter_grad: buffers");
  const Rccl& r = rccl();
  CLIPMI_RCCL(r);
  const int e = r.reduce_scatter(global, local, (size_t)count, dtype_code(dtype), kSum, (Comm)comm,
                                 (hipStream_t)stream);
  if (e) return rccl_fail(r, e, "ncclReduceScatter");
  return CLIPMI_OK;
}

extern "C" int clipmi_allreduce_grads(void* stream, void* comm, float* grads, int64_t count) {
  return clipmi_allreduce(stream, comm, CLIPMI_F32, grads, count);
}

// in-place sum over the ranks of an fp32 or bf16 buffer (bf16: the optional half-size gradient buckets)
extern "C" int clipmi_allreduce(void* stream, void* comm, int dtype, void* buf, int64_t count) {
  CLIPMI_REQUIRE(comm && count >= 0 && (dtype == CLIPMI_F32 || dtype == CLIPMI_BF16), "allreduce: args");
  if (count == 0) return CLIPMI_OK;
  CLIPMI_REQUIRE(buf, "allreduce: buffer");
  const Rccl& r = rccl();
  CLIPMI_RCCL(r);
  const int e = r.all_reduce(buf, buf, (size_t)count, dtype_code(dtype), kSum, (Comm)comm, (hipStream_t)stream);
  if (e) return rccl_fail(r, e, "ncclAllReduce");
  return CLIPMI_OK;
}

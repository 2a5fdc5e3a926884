// Data-parallel collectives of the C ABI (include/asr.h, asr_dist_*): one RCCL
// communicator per process (one process per GPU), over xGMI on one node.
//
// The reference is single-device (experiments_antisymmetric_resnet_v6.ipynb:361,
// "Default GPU Device: /device:GPU:0"); the per-step gradient all-reduce is the
// exchange step SURVEY.md §8(e) adds: the batch is split by image (no
// BatchNorm, batch-mean loss, training/training.py:295), so after each
// backward the flat fp32 gradient buffer is summed over ranks and the
// replicated Adam update applies it scaled by 1/world.
//
// librccl is opened at run time (dlopen, RTLD_LOCAL) rather than linked: the
// process may already hold PyTorch's bundled librccl, and the soname lookup
// then reuses that one instead of mapping a second copy.  Only the rccl.h
// types are used at compile time.
#include <dlfcn.h>
#include <string.h>
#include <rccl/rccl.h>

#include <mutex>

#include "asr_common.h"

namespace asr {
namespace {

struct Rccl {
  void* handle = nullptr;
  ncclResult_t (*get_unique_id)(ncclUniqueId*) = nullptr;
  ncclResult_t (*comm_init_rank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*all_reduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t,
                             hipStream_t) = nullptr;
  ncclResult_t (*broadcast)(const void*, void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
  ncclResult_t (*async_error)(ncclComm_t, ncclResult_t*) = nullptr;
  const char* (*error_string)(ncclResult_t) = nullptr;
};

Rccl g_rccl;
ncclComm_t g_comm = nullptr;
int g_rank = -1, g_world = 0;
std::mutex g_mu;

int load_rccl() {
  if (g_rccl.handle) return ASR_OK;
  // PyTorch's bundled copy is named librccl.so; ROCm's is librccl.so.1
  const char* names[] = {"librccl.so", "librccl.so.1", "/opt/rocm/lib/librccl.so.1"};
  void* h = nullptr;
  for (const char* n : names)
    if ((h = dlopen(n, RTLD_NOW | RTLD_LOCAL)) != nullptr) break;
  if (!h) return fail(ASR_E_UNSUPPORTED, "asr_dist: cannot open librccl (%s)", dlerror());
  Rccl r;
  r.handle = h;
#define ASR_SYM(field, name)                                                      \
  r.field = reinterpret_cast<decltype(r.field)>(dlsym(h, name));                  \
  if (!r.field) return fail(ASR_E_UNSUPPORTED, "asr_dist: librccl lacks %s", name)
  ASR_SYM(get_unique_id, "ncclGetUniqueId");
  ASR_SYM(comm_init_rank, "ncclCommInitRank");
  ASR_SYM(all_reduce, "ncclAllReduce");
  ASR_SYM(broadcast, "ncclBroadcast");
  ASR_SYM(comm_destroy, "ncclCommDestroy");
  ASR_SYM(async_error, "ncclCommGetAsyncError");
  ASR_SYM(error_string, "ncclGetErrorString");
#undef ASR_SYM
  g_rccl = r;
  return ASR_OK;
}

int rccl_check(ncclResult_t r, const char* what) {
  if (r == ncclSuccess) return ASR_OK;
  return fail(ASR_E_HIP, "%s: RCCL error %d (%s)", what, (int)r, g_rccl.error_string ? g_rccl.error_string(r) : "?");
}

int dtype_of(int dtype, ncclDataType_t* t) {
  switch (dtype) {
    case ASR_F32: *t = ncclFloat32; return ASR_OK;
    case ASR_BF16: *t = ncclBfloat16; return ASR_OK;
  }
  return fail(ASR_E_ARG, "asr_dist: bad dtype %d", dtype);
}

int need_comm(const char* fn) {
  if (!g_comm) return fail(ASR_E_ARG, "%s: asr_dist_init has not been called", fn);
  // a failed peer surfaces here instead of as a hang in the next collective
  ncclResult_t ae = ncclSuccess;
  ASR_TRY(rccl_check(g_rccl.async_error(g_comm, &ae), "ncclCommGetAsyncError"));
  return rccl_check(ae, fn);
}

}  // namespace
}  // namespace asr

using namespace asr;

extern "C" {

int asr_dist_unique_id(void* out) {
  if (!out) return fail(ASR_E_ARG, "asr_dist_unique_id: null output");
  std::lock_guard<std::mutex> lk(g_mu);
  ASR_TRY(load_rccl());
  ncclUniqueId id;
  ASR_TRY(rccl_check(g_rccl.get_unique_id(&id), "ncclGetUniqueId"));
  memcpy(out, id.internal, ASR_DIST_UNIQUE_ID_BYTES);
  return ASR_OK;
}

int asr_dist_init(int rank, int world, const void* unique_id) {
  static_assert(ASR_DIST_UNIQUE_ID_BYTES == NCCL_UNIQUE_ID_BYTES, "unique id size");
  if (!unique_id || world < 1 || rank < 0 || rank >= world)
    return fail(ASR_E_ARG, "asr_dist_init: bad arguments (rank %d, world %d)", rank, world);
  std::lock_guard<std::mutex> lk(g_mu);
  if (g_comm) return fail(ASR_E_ARG, "asr_dist_init: already initialised (rank %d of %d)", g_rank, g_world);
  ASR_TRY(load_rccl());
  ncclUniqueId id;
  memcpy(id.internal, unique_id, ASR_DIST_UNIQUE_ID_BYTES);
  ncclComm_t c = nullptr;
  ASR_TRY(rccl_check(g_rccl.comm_init_rank(&c, world, id, rank), "ncclCommInitRank"));
  g_comm = c;
  g_rank = rank;
  g_world = world;
  return ASR_OK;
}

int asr_dist_allreduce_sum(void* buf, size_t count, int dtype, asr_stream_t stream) {
  if (!buf && count) return fail(ASR_E_ARG, "asr_dist_allreduce_sum: null buffer");
  ASR_TRY(need_comm("asr_dist_allreduce_sum"));
  ncclDataType_t t;
  ASR_TRY(dtype_of(dtype, &t));
  if (count == 0) return ASR_OK;
  return rccl_check(g_rccl.all_reduce(buf, buf, count, t, ncclSum, g_comm, (hipStream_t)stream), "ncclAllReduce");
}

int asr_dist_broadcast(void* buf, size_t count, int dtype, int root, asr_stream_t stream) {
  if (!buf && count) return fail(ASR_E_ARG, "asr_dist_broadcast: null buffer");
  ASR_TRY(need_comm("asr_dist_broadcast"));
  if (root < 0 || root >= g_world) return fail(ASR_E_ARG, "asr_dist_broadcast: bad root %d", root);
  ncclDataType_t t;
  ASR_TRY(dtype_of(dtype, &t));
  if (count == 0) return ASR_OK;
  return rccl_check(g_rccl.broadcast(buf, buf, count, t, root, g_comm, (hipStream_t)stream), "ncclBroadcast");
}

int asr_dist_world_size(void) { return g_comm ? g_world : 0; }

int asr_dist_finalize(void) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (!g_comm) return ASR_OK;
  ncclComm_t c = g_comm;
  g_comm = nullptr;
  g_rank = -1;
  g_world = 0;
  return rccl_check(g_rccl.comm_destroy(c), "ncclCommDestroy");
}

}  // extern "C"

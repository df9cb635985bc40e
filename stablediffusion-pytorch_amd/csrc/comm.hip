// Gradient all-reduce through RCCL, issued by the library itself.
//
// The data-parallel reducer's bucket all-reduces used to go through torch.distributed (ProcessGroupNCCL): each one a
// Python callout out of the native plan replay, run on the process group's internal stream. That stream is bound to
// one of the process's four hardware queues at its first use, after the engines' streams, and so shares a queue with
// one of them (sdmi/streams.py) -- a collective waiting on that queue holds up a weight-gradient or compute stream.
// Here the library owns an RCCL communicator and issues ncclAllReduce on the caller's stream (the reducer's), so the
// collective runs on the reducer's queue, and a recording plan keeps it as a native op replayed without Python.
// RCCL is bound at run time (dlopen of the librccl.so the process already has: torch's), libsdmi.so does not link it.
#include <dlfcn.h>
#include <rccl/rccl.h>

#include <cstring>

#include "../../include/sdmi.h"
#include "launch.h"

namespace sdmi_rt {
namespace {

struct Rccl {
  void* handle = nullptr;
  decltype(&ncclGetUniqueId) get_unique_id = nullptr;
  decltype(&ncclCommInitRank) comm_init_rank = nullptr;
  decltype(&ncclAllReduce) all_reduce = nullptr;
  decltype(&ncclCommDestroy) comm_destroy = nullptr;
};
Rccl g_rccl;

template <typename F>
bool bind(F& f, const char* name) {
  f = (F)dlsym(g_rccl.handle, name);
  return f != nullptr;
}

}  // namespace

int issue_allreduce(void* comm, void* buf, size_t count, int dtype, hipStream_t stream) {
  if (!g_rccl.all_reduce) return -10;
  const ncclDataType_t dt = dtype == 1 ? ncclBfloat16 : ncclFloat32;
  const ncclResult_t r = g_rccl.all_reduce(buf, buf, count, dt, ncclSum, (ncclComm_t)comm, stream);
  return r == ncclSuccess ? 0 : 1000 + (int)r;
}

}  // namespace sdmi_rt

using sdmi_rt::g_rccl;

extern "C" int sdmi_comm_load(const char* rccl_path) {
  if (g_rccl.all_reduce) return 0;
  if (!rccl_path) return -1;
  g_rccl.handle = dlopen(rccl_path, RTLD_NOW | RTLD_LOCAL);
  if (!g_rccl.handle) return -2;
  if (!sdmi_rt::bind(g_rccl.get_unique_id, "ncclGetUniqueId") ||
      !sdmi_rt::bind(g_rccl.comm_init_rank, "ncclCommInitRank") ||
      !sdmi_rt::bind(g_rccl.comm_destroy, "ncclCommDestroy") || !sdmi_rt::bind(g_rccl.all_reduce, "ncclAllReduce")) {
    g_rccl.all_reduce = nullptr;
    return -3;
  }
  return 0;
}

extern "C" int sdmi_comm_unique_id(unsigned char* id) {
  if (!id) return -1;
  if (!g_rccl.get_unique_id) return -10;
  ncclUniqueId u;
  const ncclResult_t r = g_rccl.get_unique_id(&u);
  if (r != ncclSuccess) return 1000 + (int)r;
  memcpy(id, u.internal, NCCL_UNIQUE_ID_BYTES);
  return 0;
}

extern "C" int sdmi_comm_init(const unsigned char* id, int nranks, int rank, void** comm) {
  if (!id || !comm || nranks < 1 || rank < 0 || rank >= nranks) return -1;
  if (!g_rccl.comm_init_rank) return -10;
  ncclUniqueId u;
  memcpy(u.internal, id, NCCL_UNIQUE_ID_BYTES);
  ncclComm_t c = nullptr;
  const ncclResult_t r = g_rccl.comm_init_rank(&c, nranks, u, rank);
  if (r != ncclSuccess) return 1000 + (int)r;
  *comm = (void*)c;
  return 0;
}

extern "C" int sdmi_allreduce(void* comm, void* buf, long long count, int dtype, sdmi_stream_t stream) {
  if (!comm || !buf || count < 0 || (dtype != 0 && dtype != 1)) return -1;
  if (count == 0) return 0;
  if (sdmi_rt::g_recording) sdmi_rt::record_allreduce(comm, buf, (size_t)count, dtype, (hipStream_t)stream);
  return sdmi_rt::issue_allreduce(comm, buf, (size_t)count, dtype, (hipStream_t)stream);
}

extern "C" int sdmi_comm_destroy(void* comm) {
  if (!comm) return -1;
  if (!g_rccl.comm_destroy) return -10;
  const ncclResult_t r = g_rccl.comm_destroy((ncclComm_t)comm);
  return r == ncclSuccess ? 0 : 1000 + (int)r;
}

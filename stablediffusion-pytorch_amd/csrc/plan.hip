// Native launch plans: a training step recorded once and re-issued from C++.
//
// While a plan records (sdmi_plan_begin .. sdmi_plan_end) the step runs for real; every kernel launch of the library
// (launch.h) is appended with its marshalled arguments, and the host layer notes the stream / event edges it issues
// (sdmi_plan_note_event / sdmi_plan_note_wait) and the points where it must run something the library does not
// own -- an RCCL collective, a torch copy -- as numbered callouts (sdmi_plan_note_callout). sdmi_plan_replay then
// re-issues the ops in recorded order, same pointers, grids and streams, until the next callout (returned to the
// caller, who runs it and resumes) or the end. Per launch this costs one hipLaunchKernel: no Python, no ctypes
// marshalling, no GEMM planning (split / tile choice, descriptor validation) on the replay path.
#include <cstring>
#include <memory>
#include <new>
#include <vector>

#include "../../include/sdmi.h"
#include "launch.h"

namespace sdmi_rt {

void* g_recording = nullptr;

namespace {

enum OpKind { OP_LAUNCH = 0, OP_EVENT = 1, OP_WAIT = 2, OP_CALLOUT = 3, OP_ALLREDUCE = 4 };

struct alignas(16) Chunk16 {
  unsigned char b[16];
};

struct Op {
  int kind;
  const void* fn = nullptr;
  dim3 grid, block;
  unsigned shmem = 0;
  hipStream_t stream = nullptr;
  hipEvent_t event = nullptr;
  int callout = -1;
  void* comm = nullptr;  // OP_ALLREDUCE: communicator, buffer, element count, dtype (0 fp32, 1 bf16)
  void* buf = nullptr;
  size_t count = 0;
  int dtype = 0;
  std::vector<Chunk16> args;   // copy of the argument tuple (16-B aligned)
  std::vector<unsigned> offs;  // byte offset of each argument inside it
};

struct Plan {
  std::vector<Op> ops;
  int launches = 0;
  std::vector<void*> scratch;  // argument pointer array reused by replay
};

}  // namespace

void record_launch(const void* fn, dim3 grid, dim3 block, unsigned shmem, hipStream_t stream, const void* args,
                   size_t bytes, const unsigned* offsets, int nargs) {
  Plan* p = (Plan*)g_recording;
  Op op;
  op.kind = OP_LAUNCH;
  op.fn = fn;
  op.grid = grid;
  op.block = block;
  op.shmem = shmem;
  op.stream = stream;
  op.args.resize((bytes + 15) / 16);
  if (bytes) memcpy(op.args.data(), args, bytes);
  op.offs.assign(offsets, offsets + nargs);
  if ((int)p->scratch.size() < nargs) p->scratch.resize(nargs);
  p->ops.push_back(std::move(op));
  ++p->launches;
}

void record_allreduce(void* comm, void* buf, size_t count, int dtype, hipStream_t stream) {
  Plan* p = (Plan*)g_recording;
  Op op;
  op.kind = OP_ALLREDUCE;
  op.comm = comm;
  op.buf = buf;
  op.count = count;
  op.dtype = dtype;
  op.stream = stream;
  p->ops.push_back(std::move(op));
}

}  // namespace sdmi_rt

using sdmi_rt::Plan;

extern "C" int sdmi_plan_begin(void) {
  if (sdmi_rt::g_recording) return -1;  // not re-entrant
  sdmi_rt::g_recording = new (std::nothrow) Plan();
  return sdmi_rt::g_recording ? 0 : -2;
}

extern "C" int sdmi_plan_end(void** plan) {
  if (!plan || !sdmi_rt::g_recording) return -1;
  *plan = sdmi_rt::g_recording;
  sdmi_rt::g_recording = nullptr;
  return 0;
}

extern "C" int sdmi_plan_recording(void) { return sdmi_rt::g_recording != nullptr; }

extern "C" int sdmi_plan_note_event(void* event, sdmi_stream_t stream) {
  Plan* p = (Plan*)sdmi_rt::g_recording;
  if (!p) return 0;
  if (!event) return -1;
  sdmi_rt::Op op;
  op.kind = sdmi_rt::OP_EVENT;
  op.event = (hipEvent_t)event;
  op.stream = (hipStream_t)stream;
  p->ops.push_back(std::move(op));
  return 0;
}

extern "C" int sdmi_plan_note_wait(sdmi_stream_t stream, void* event) {
  Plan* p = (Plan*)sdmi_rt::g_recording;
  if (!p) return 0;
  if (!event) return -1;
  sdmi_rt::Op op;
  op.kind = sdmi_rt::OP_WAIT;
  op.event = (hipEvent_t)event;
  op.stream = (hipStream_t)stream;
  p->ops.push_back(std::move(op));
  return 0;
}

extern "C" int sdmi_plan_note_callout(int id) {
  Plan* p = (Plan*)sdmi_rt::g_recording;
  if (!p) return 0;
  sdmi_rt::Op op;
  op.kind = sdmi_rt::OP_CALLOUT;
  op.callout = id;
  p->ops.push_back(std::move(op));
  return 0;
}

extern "C" int sdmi_plan_info(const void* plan, int* ops, int* launches) {
  const Plan* p = (const Plan*)plan;
  if (!p) return -1;
  if (ops) *ops = (int)p->ops.size();
  if (launches) *launches = p->launches;
  return 0;
}

extern "C" int sdmi_plan_replay(void* plan, int start, int* callout, int* next) {
  Plan* p = (Plan*)plan;
  if (!p || start < 0 || !callout || !next) return -1;
  void** ptrs = p->scratch.data();
  const int n = (int)p->ops.size();
  for (int i = start; i < n; ++i) {
    const sdmi_rt::Op& op = p->ops[i];
    hipError_t e = hipSuccess;
    switch (op.kind) {
      case sdmi_rt::OP_LAUNCH: {
        const unsigned char* base = (const unsigned char*)op.args.data();
        for (size_t a = 0; a < op.offs.size(); ++a) ptrs[a] = (void*)(base + op.offs[a]);
        e = hipLaunchKernel(op.fn, op.grid, op.block, ptrs, op.shmem, op.stream);
        break;
      }
      case sdmi_rt::OP_EVENT: e = hipEventRecord(op.event, op.stream); break;
      case sdmi_rt::OP_WAIT: e = hipStreamWaitEvent(op.stream, op.event, 0); break;
      case sdmi_rt::OP_ALLREDUCE: {
        const int rc = sdmi_rt::issue_allreduce(op.comm, op.buf, op.count, op.dtype, op.stream);
        if (rc != 0) {
          *callout = -1;
          *next = i;
          return rc;
        }
        break;
      }
      default:
        *callout = op.callout;
        *next = i + 1;
        return 0;
    }
    if (e != hipSuccess) {
      *callout = -1;
      *next = i;
      return (int)e;
    }
  }
  *callout = -1;
  *next = n;
  return 0;
}

// the stream an op was recorded on (launches, event records, waits, all-reduces; nullptr for callouts)
extern "C" int sdmi_plan_op_stream(const void* plan, int i, sdmi_stream_t* stream) {
  const Plan* p = (const Plan*)plan;
  if (!p || i < 0 || i >= (int)p->ops.size() || !stream) return -1;
  *stream = (sdmi_stream_t)p->ops[i].stream;
  return 0;
}

// Per-op inspection for profiling tools (scripts/plan_profile.py): op kind (0 launch, 1 event record, 2 stream wait,
// 3 callout, 4 all-reduce), kernel name, grid / block, LDS bytes.
extern "C" int sdmi_plan_op_info(const void* plan, int i, int* kind, const char** name, int* grid, int* block,
                                 int* shmem) {
  const Plan* p = (const Plan*)plan;
  if (!p || i < 0 || i >= (int)p->ops.size()) return -1;
  const sdmi_rt::Op& op = p->ops[i];
  if (kind) *kind = op.kind;
  if (name) *name = op.kind == sdmi_rt::OP_LAUNCH ? hipKernelNameRefByPtr(op.fn, op.stream) : nullptr;
  if (grid) {
    grid[0] = (int)op.grid.x;
    grid[1] = (int)op.grid.y;
    grid[2] = (int)op.grid.z;
  }
  if (block) *block = (int)(op.block.x * op.block.y * op.block.z);
  if (shmem) *shmem = (int)op.shmem;
  return 0;
}

// Re-issue launch op i alone `iters` times on its stream between two events (after `warm` untimed issues) and
// return the average device time in microseconds. The plan's buffers are live (private pool), so the op reads and
// writes exactly the memory it does inside the step (in-place accumulating ops change values; timing only).
extern "C" int sdmi_plan_time_op(void* plan, int i, int warm, int iters, float* us) {
  Plan* p = (Plan*)plan;
  if (!p || i < 0 || i >= (int)p->ops.size() || iters < 1 || !us) return -1;
  const sdmi_rt::Op& op = p->ops[i];
  if (op.kind != sdmi_rt::OP_LAUNCH) return -2;
  void** ptrs = p->scratch.data();
  const unsigned char* base = (const unsigned char*)op.args.data();
  for (size_t a = 0; a < op.offs.size(); ++a) ptrs[a] = (void*)(base + op.offs[a]);
  hipEvent_t e0, e1;
  if (hipEventCreate(&e0) != hipSuccess) return -3;
  if (hipEventCreate(&e1) != hipSuccess) return -3;
  hipError_t e = hipSuccess;
  for (int w = 0; w < warm && e == hipSuccess; ++w) e = hipLaunchKernel(op.fn, op.grid, op.block, ptrs, op.shmem, op.stream);
  if (e == hipSuccess) e = hipEventRecord(e0, op.stream);
  for (int r = 0; r < iters && e == hipSuccess; ++r) e = hipLaunchKernel(op.fn, op.grid, op.block, ptrs, op.shmem, op.stream);
  if (e == hipSuccess) e = hipEventRecord(e1, op.stream);
  if (e == hipSuccess) e = hipEventSynchronize(e1);
  float ms = 0.f;
  if (e == hipSuccess) e = hipEventElapsedTime(&ms, e0, e1);
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  if (e != hipSuccess) return (int)e;
  *us = ms * 1000.f / (float)iters;
  return 0;
}

extern "C" int sdmi_plan_destroy(void* plan) {
  delete (Plan*)plan;
  return 0;
}

// Kernel launch helper of libsdmi: every kernel of the library is launched through sdmi_rt::launch, which issues
// it with hipLaunchKernel and -- while a launch plan is being recorded (plan.hip, sdmi_plan_begin) -- appends the
// launch (kernel, grid, block, LDS bytes, stream, a copy of the marshalled arguments) to the plan, so a training
// step recorded once can be re-issued from C++ without the Python / ctypes / host-planning cost per launch.
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <tuple>
#include <type_traits>
#include <utility>

namespace sdmi_rt {

// non-null while a plan records (one host thread issues a step; the recorder is not re-entrant)
extern void* g_recording;

void record_launch(const void* fn, dim3 grid, dim3 block, unsigned shmem, hipStream_t stream, const void* args,
                   size_t bytes, const unsigned* offsets, int nargs);

// in-place sum all-reduce through the library's RCCL communicator (comm.hip); the plan records and replays it
void record_allreduce(void* comm, void* buf, size_t count, int dtype, hipStream_t stream);
int issue_allreduce(void* comm, void* buf, size_t count, int dtype, hipStream_t stream);

template <typename Tuple, size_t... I>
inline void arg_ptrs(Tuple& t, void** ptrs, unsigned* offs, std::index_sequence<I...>) {
  ((ptrs[I] = (void*)&std::get<I>(t), offs[I] = (unsigned)((const char*)&std::get<I>(t) - (const char*)&t)), ...);
}

template <typename... P, typename... A>
inline hipError_t launch(void (*kernel)(P...), dim3 grid, dim3 block, size_t shmem, hipStream_t stream, A&&... a) {
  static_assert(sizeof...(P) == sizeof...(A), "kernel argument count");
  using T = std::tuple<std::decay_t<P>...>;
  static_assert((std::is_trivially_copyable<std::decay_t<P>>::value && ...), "kernel arguments must be plain data");
  T args(std::forward<A>(a)...);
  constexpr size_t n = sizeof...(P);
  void* ptrs[n > 0 ? n : 1];
  unsigned offs[n > 0 ? n : 1];
  arg_ptrs(args, ptrs, offs, std::index_sequence_for<P...>{});
  const hipError_t e = hipLaunchKernel((const void*)kernel, grid, block, ptrs, shmem, stream);
  if (g_recording && e == hipSuccess)
    record_launch((const void*)kernel, grid, block, (unsigned)shmem, stream, &args, sizeof(T), offs, (int)n);
  return e;
}

}  // namespace sdmi_rt

// The one exchange step of the T-sharded path. Every statistic a pass
// produces is a sum over t (src/core.rs:76,218,226,274; src/whitening.rs:25), so each
// pass of a rank ends with ONE in-place sum-all-reduce of its packed fp64 statistics.
//
// Two implementations sit behind DeviceCtx:
//   * RCCL over xGMI — one process per GPU (bench.py --gpus N). A cross-process abort
//     word in POSIX shared memory lets a failing rank end every peer's wait: the peers
//     poll their stream instead of blocking in hipStreamSynchronize, and on the abort
//     word (or a dead peer process, or the watchdog timeout) call ncclCommAbort and raise.
//   * an in-process group — `world` contexts in one process, one host thread per rank
//     (all may share one GPU). allreduce copies the rank's statistics to host memory,
//     meets the other ranks at a barrier and adds the rank buffers in fixed rank order,
//     so every rank gets identical bits. Each call also compares a call-site tag and
//     length across ranks: ranks that diverge (different collectives in the same slot)
//     raise instead of summing unrelated buffers. This runs the rank-replicated solver
//     and every communicator branch of DeviceCtx on a single-GPU box.
#pragma once
#include <hip/hip_runtime_api.h>

#include <cstdint>
#include <memory>
#include <string>

namespace pcamd {

class Collective {
 public:
  virtual ~Collective() = default;
  virtual int rank() const = 0;
  virtual int world() const = 0;
  // in-place Σ over the ranks of n doubles at device pointer d, ordered after the work
  // already on `stream`; `tag` names the call site (checked across ranks where possible)
  virtual void allreduce(double* d, size_t n, hipStream_t stream, const char* tag) = 0;
  // return once `stream` has drained; raise if the group was aborted meanwhile
  virtual void wait(hipStream_t stream) = 0;
  // this rank failed: every rank's pending and later collectives end with an error
  virtual void abort(const std::string& why) noexcept = 0;
  virtual bool aborted() const = 0;
  virtual const char* kind() const = 0;
  uint64_t n_allreduce = 0;
};

struct LocalGroup;  // shared state of an in-process rank group
std::shared_ptr<LocalGroup> make_local_group(int world);
int local_group_world(const LocalGroup& g);
std::unique_ptr<Collective> make_local_collective(std::shared_ptr<LocalGroup> g, int rank);
// uid: the 128-byte ncclUniqueId broadcast by the caller
std::unique_ptr<Collective> make_rccl_collective(int rank, int world, const char* uid);
int rccl_unique_id(char* out);

}  // namespace pcamd

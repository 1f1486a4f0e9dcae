// Collective implementations behind DeviceCtx (collective.hpp): RCCL with a
// cross-process abort word, and the in-process rank group.
#include "collective.hpp"

#include <fcntl.h>
#include <rccl/rccl.h>
#include <sched.h>
#include <signal.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <atomic>
#include <cerrno>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <vector>

#include "evaluator.hpp"

namespace pcamd {
namespace {

#define CHK_HIP(expr)                                                                      \
  do {                                                                                     \
    hipError_t e_ = (expr);                                                                \
    if (e_ != hipSuccess)                                                                  \
      throw computation_error(std::string("HIP: ") + hipGetErrorString(e_) + " at " #expr); \
  } while (0)

using Clock = std::chrono::steady_clock;

// watchdog: a collective that has not completed after this long ends the group
// (PICARD_COMM_TIMEOUT_S, default 600 s; a C3 pass takes milliseconds)
double comm_timeout_s() {
  const char* e = std::getenv("PICARD_COMM_TIMEOUT_S");
  const double v = e ? std::atof(e) : 0.0;
  return v > 0.0 ? v : 600.0;
}

double secs_since(Clock::time_point t0) { return std::chrono::duration<double>(Clock::now() - t0).count(); }

// ---------------------------------------------------------------------------
// In-process group
// ---------------------------------------------------------------------------
}  // namespace

struct LocalGroup {
  explicit LocalGroup(int w) : world(w), slot(w), tag(w) {}
  const int world;
  std::mutex mu;
  std::condition_variable cv;
  int arrived = 0;
  uint64_t gen = 0;
  bool aborted = false;
  std::string why;
  std::vector<std::vector<double>> slot;  // each rank's contribution to the current all-reduce
  std::vector<std::string> tag;           // … and the call site it came from

  void abort(const std::string& m) {
    std::lock_guard<std::mutex> lk(mu);
    if (!aborted) {
      aborted = true;
      why = m;
    }
    cv.notify_all();
  }
  [[noreturn]] void raise_aborted() {
    throw computation_error("rank group aborted: " + why);
  }
  // all `world` ranks meet; raises once the group is aborted or the watchdog fires
  void barrier(double timeout_s) {
    std::unique_lock<std::mutex> lk(mu);
    if (aborted) raise_aborted();
    const uint64_t my = gen;
    if (++arrived == world) {
      arrived = 0;
      ++gen;
      cv.notify_all();
      return;
    }
    const auto t0 = Clock::now();
    while (gen == my && !aborted) {
      cv.wait_for(lk, std::chrono::milliseconds(100));
      if (gen == my && !aborted && secs_since(t0) > timeout_s) {
        aborted = true;
        why = "collective timed out (PICARD_COMM_TIMEOUT_S) waiting for the other ranks";
        cv.notify_all();
      }
    }
    if (aborted) raise_aborted();
  }
};

std::shared_ptr<LocalGroup> make_local_group(int world) {
  if (world < 1) throw invalid_dimensions("rank group: world_size must be >= 1");
  return std::make_shared<LocalGroup>(world);
}
int local_group_world(const LocalGroup& g) { return g.world; }

namespace {

class LocalCollective final : public Collective {
 public:
  LocalCollective(std::shared_ptr<LocalGroup> g, int rank) : g_(std::move(g)), rank_(rank), timeout_(comm_timeout_s()) {
    if (rank < 0 || rank >= g_->world) throw invalid_dimensions("rank group: rank out of range");
  }
  int rank() const override { return rank_; }
  int world() const override { return g_->world; }
  const char* kind() const override { return "local"; }
  bool aborted() const override {
    std::lock_guard<std::mutex> lk(g_->mu);
    return g_->aborted;
  }
  void abort(const std::string& why) noexcept override {
    try {
      g_->abort("rank " + std::to_string(rank_) + ": " + why);
    } catch (...) {
    }
  }
  void allreduce(double* d, size_t n, hipStream_t stream, const char* tag) override {
    if (aborted()) g_->raise_aborted();
    std::vector<double>& mine = g_->slot[rank_];
    mine.resize(n);
    g_->tag[rank_] = tag ? tag : "";
    if (n) CHK_HIP(hipMemcpyAsync(mine.data(), d, n * sizeof(double), hipMemcpyDeviceToHost, stream));
    CHK_HIP(hipStreamSynchronize(stream));
    g_->barrier(timeout_);  // every rank's buffer is in place
    for (int r = 0; r < g_->world; ++r)
      if (g_->slot[r].size() != n || g_->tag[r] != g_->tag[rank_]) {
        const std::string m = "ranks diverged: rank " + std::to_string(rank_) + " issued all-reduce '" +
                              g_->tag[rank_] + "' of " + std::to_string(n) + " values, rank " + std::to_string(r) +
                              " '" + g_->tag[r] + "' of " + std::to_string(g_->slot[r].size());
        g_->abort(m);
        g_->raise_aborted();
      }
    // fixed rank order: every rank forms the same sum, bit for bit
    sum_.assign(n, 0.0);
    for (int r = 0; r < g_->world; ++r) {
      const double* s = g_->slot[r].data();
      for (size_t i = 0; i < n; ++i) sum_[i] += s[i];
    }
    if (n) CHK_HIP(hipMemcpyAsync(d, sum_.data(), n * sizeof(double), hipMemcpyHostToDevice, stream));
    ++n_allreduce;
    g_->barrier(timeout_);  // every rank has read the buffers: they may be reused
  }
  void wait(hipStream_t stream) override {
    CHK_HIP(hipStreamSynchronize(stream));
    if (aborted()) g_->raise_aborted();
  }

 private:
  std::shared_ptr<LocalGroup> g_;
  const int rank_;
  const double timeout_;
  std::vector<double> sum_;  // the reduced values; alive until the next call's synchronisation
};

// ---------------------------------------------------------------------------
// RCCL with a cross-process abort word
// ---------------------------------------------------------------------------
constexpr int kMaxRanks = 64;
struct AbortWord {
  std::atomic<int> failed;  // 0 = healthy, r + 1 = rank r raised
  char why[256];
  int32_t pid[kMaxRanks];
};

class RcclCollective final : public Collective {
 public:
  RcclCollective(int rank, int world, const char* uid) : rank_(rank), world_(world), timeout_(comm_timeout_s()) {
    ncclUniqueId id;
    std::memcpy(&id, uid, sizeof id);
    open_abort_word(uid);
    const ncclResult_t r = ncclCommInitRank(&comm_, world, id, rank);
    // ncclCommInitRank is collective and every rank maps the word before calling it, so once
    // it returns (either way) the name is no longer needed: every rank unlinks it (ENOENT is
    // fine), which also covers the other nodes of a multi-node group and a failed init
    if (!shm_name_.empty()) shm_unlink(shm_name_.c_str());
    if (r != ncclSuccess) {
      close_abort_word();
      throw computation_error(std::string("RCCL: ") + ncclGetErrorString(r) + " at ncclCommInitRank");
    }
  }
  ~RcclCollective() override {
    if (comm_) (void)ncclCommDestroy(comm_);
    close_abort_word();
  }
  int rank() const override { return rank_; }
  int world() const override { return world_; }
  const char* kind() const override { return "rccl"; }
  bool aborted() const override { return local_aborted_.load() || (aw_ && aw_->failed.load() != 0); }

  // May be called from any thread (pc_ctx_abort from a watchdog while the fit thread is in
  // allreduce / wait): comm_ and the reason are guarded by mu_, the flag is atomic.
  void abort(const std::string& why) noexcept override {
    if (aw_) {
      int expect = 0;
      if (aw_->failed.compare_exchange_strong(expect, rank_ + 1)) {
        const std::string m = "rank " + std::to_string(rank_) + ": " + why;
        std::strncpy(aw_->why, m.c_str(), sizeof aw_->why - 1);
        aw_->why[sizeof aw_->why - 1] = 0;
      }
    }
    std::lock_guard<std::mutex> lk(mu_);
    if (local_why_.empty()) {
      try {
        local_why_ = why;
      } catch (...) {
      }
    }
    local_aborted_.store(true);
    if (comm_) {
      (void)ncclCommAbort(comm_);  // ends this rank's in-flight collectives
      comm_ = nullptr;
    }
  }

  void allreduce(double* d, size_t n, hipStream_t stream, const char* tag) override {
    (void)tag;
    check();
    ncclResult_t r;
    {
      std::lock_guard<std::mutex> lk(mu_);
      if (!comm_) throw computation_error("rank group aborted: " + local_why_);
      r = ncclAllReduce(d, d, n, ncclFloat64, ncclSum, comm_, stream);
    }
    if (r != ncclSuccess) {
      const std::string m = std::string("RCCL: ") + ncclGetErrorString(r) + " in ncclAllReduce";
      abort(m);
      throw computation_error(m);
    }
    ++n_allreduce;
  }

  // Poll instead of blocking in hipStreamSynchronize: a peer that raised (abort word),
  // died (its pid is gone), an RCCL async error or the watchdog ends the wait.
  void wait(hipStream_t stream) override {
    const auto t0 = Clock::now();
    auto last_probe = t0;
    for (uint64_t spin = 0;; ++spin) {
      const hipError_t e = hipStreamQuery(stream);
      if (e == hipSuccess) break;
      if (e != hipErrorNotReady) {
        (void)hipGetLastError();
        const std::string m = std::string("HIP: ") + hipGetErrorString(e) + " while waiting for a collective";
        abort(m);
        throw computation_error(m);
      }
      check();
      const auto now = Clock::now();
      if (std::chrono::duration<double>(now - last_probe).count() > 0.1) {
        last_probe = now;
        probe(secs_since(t0));
      }
      // yield between probes while a pass can still be running (C3's longest shard pass is
      // ≈ 10 ms at 8 ranks, 75 ms at 1); a usleep wakes 20–70 µs late, a cost every pass paid
      // once the old cap of 4096 yields (a few ms) was spent. Past 0.5 s (a slow peer) sleep.
      if (spin < 1024 || secs_since(t0) < 0.5) sched_yield();
      else usleep(20);
    }
    check();
  }

 private:
  void check() {
    if (local_aborted_.load()) {
      std::lock_guard<std::mutex> lk(mu_);
      throw computation_error("rank group aborted: " + local_why_);
    }
    if (aw_ && aw_->failed.load() != 0) {
      const std::string m = std::string(aw_->why);
      abort(m);
      throw computation_error("rank group aborted: " + m);
    }
  }
  // RCCL async error, dead peer processes, watchdog
  void probe(double waited_s) {
    ncclResult_t ae = ncclSuccess;
    bool failed;
    {
      std::lock_guard<std::mutex> lk(mu_);
      failed = comm_ && ncclCommGetAsyncError(comm_, &ae) == ncclSuccess && ae != ncclSuccess && ae != ncclInProgress;
    }
    if (failed) {
      const std::string m = std::string("RCCL async error: ") + ncclGetErrorString(ae);
      abort(m);
      throw computation_error(m);
    }
    if (aw_)
      for (int r = 0; r < world_ && r < kMaxRanks; ++r) {
        const pid_t p = aw_->pid[r];
        if (r != rank_ && p > 0 && kill(p, 0) != 0 && errno == ESRCH) {
          const std::string m = "rank " + std::to_string(r) + " (pid " + std::to_string(p) + ") exited";
          abort(m);
          throw computation_error("rank group aborted: " + m);
        }
      }
    if (waited_s > timeout_) {
      const std::string m = "collective timed out after " + std::to_string((int)waited_s) + " s (PICARD_COMM_TIMEOUT_S)";
      abort(m);
      throw computation_error(m);
    }
  }
  void open_abort_word(const char* uid) {
    // name from the unique id: the same on every rank of this communicator only
    uint64_t h = 1469598103934665603ull;
    for (size_t i = 0; i < sizeof(ncclUniqueId); ++i) h = (h ^ (uint8_t)uid[i]) * 1099511628211ull;
    char name[64];
    std::snprintf(name, sizeof name, "/picard_grp_%016llx", (unsigned long long)h);
    const int fd = shm_open(name, O_CREAT | O_RDWR, 0600);
    if (fd < 0) {
      std::fprintf(stderr, "picard: no shared abort word (%s); a failing peer is detected by the watchdog only\n",
                   std::strerror(errno));
      return;
    }
    if (ftruncate(fd, sizeof(AbortWord)) != 0) {
      close(fd);
      shm_unlink(name);
      return;
    }
    void* p = mmap(nullptr, sizeof(AbortWord), PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    close(fd);
    if (p == MAP_FAILED) {
      shm_unlink(name);
      return;
    }
    aw_ = static_cast<AbortWord*>(p);  // zero-filled on creation: failed = 0
    if (rank_ < kMaxRanks) aw_->pid[rank_] = (int32_t)getpid();
    shm_name_ = name;
  }
  void close_abort_word() {
    if (aw_) munmap(aw_, sizeof(AbortWord));
    aw_ = nullptr;
  }

  const int rank_, world_;
  const double timeout_;
  ncclComm_t comm_ = nullptr;
  AbortWord* aw_ = nullptr;
  std::string shm_name_;
  mutable std::mutex mu_;  // comm_, local_why_
  std::atomic<bool> local_aborted_{false};
  std::string local_why_;
};

}  // namespace

std::unique_ptr<Collective> make_local_collective(std::shared_ptr<LocalGroup> g, int rank) {
  return std::unique_ptr<Collective>(new LocalCollective(std::move(g), rank));
}

std::unique_ptr<Collective> make_rccl_collective(int rank, int world, const char* uid) {
  return std::unique_ptr<Collective>(new RcclCollective(rank, world, uid));
}

int rccl_unique_id(char* out) {
  ncclUniqueId id;
  if (ncclGetUniqueId(&id) != ncclSuccess) return 1;
  std::memcpy(out, &id, sizeof id);
  return 0;
}

}  // namespace pcamd

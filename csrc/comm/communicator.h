// Native RCCL communicator: the MI355X data plane that replaces the
// reference's libipc TCP sockets + ipc.Tree b-ary tree.
//
//  reference                                    here
//  -------------------------------------------  -------------------------------------------
//  tree.allReduce(value, add)  (AllReduceSGD:12) all_reduce -> ncclAllReduce(sum) on a flat
//                                                 bucket, issued on the caller's HIP stream
//  tree.scatter(value)         (AllReduceSGD:52) broadcast -> ncclBroadcast(root)
//  client:send / client:recv   (AsyncEA:87-130)  send / recv -> ncclSend / ncclRecv (grouped)
//  ipc.server/ipc.client rendezvous             ncclUniqueId exchanged through the c10d TCPStore
//
// The communicator never synchronises the host: every call is enqueued on a
// stream handle supplied by Python (a torch stream), so calls are legal inside
// hipGraph capture and can be overlapped with compute on a side stream.
#pragma once
#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <mutex>
#include <thread>
#include <string>
#include <vector>

#include "dl_common.h"
#include "pause_gate.h"
#include "retirable.h"

#define DL_NCCL_CHECK(expr)                                                                                      \
  do {                                                                                                           \
    ncclResult_t _r = (expr);                                                                                    \
    if (_r != ncclSuccess) {                                                                                     \
      throw std::runtime_error(std::string("RCCL error: ") + ncclGetErrorString(_r) + " at " + __FILE__ + ":" + \
                               std::to_string(__LINE__));                                                        \
    }                                                                                                            \
  } while (0)

namespace dl {

// dtype codes shared with python (torch_distlearn_amd/parallel/comm.py)
enum DType : int { kF32 = 0, kBF16 = 1, kF16 = 2, kI64 = 3, kI32 = 4, kU8 = 5, kF64 = 6 };
enum ROp : int { kSum = 0, kProd = 1, kMax = 2, kMin = 3, kAvg = 4 };

inline ncclDataType_t to_nccl(int dt) {
  switch (dt) {
    case kF32: return ncclFloat32;
    case kBF16: return ncclBfloat16;
    case kF16: return ncclFloat16;
    case kI64: return ncclInt64;
    case kI32: return ncclInt32;
    case kU8: return ncclUint8;
    case kF64: return ncclFloat64;
  }
  throw std::runtime_error("unsupported dtype code " + std::to_string(dt));
}

inline ncclRedOp_t to_nccl_op(int op) {
  switch (op) {
    case kSum: return ncclSum;
    case kProd: return ncclProd;
    case kMax: return ncclMax;
    case kMin: return ncclMin;
    case kAvg: return ncclAvg;
  }
  throw std::runtime_error("unsupported reduction op " + std::to_string(op));
}

inline std::string rccl_unique_id() {
  ncclUniqueId id;
  DL_NCCL_CHECK(ncclGetUniqueId(&id));
  return std::string(reinterpret_cast<const char*>(&id), sizeof(id));
}

inline int rccl_version() {
  int v = 0;
  DL_NCCL_CHECK(ncclGetVersion(&v));
  return v;
}

// Failure detection.  RCCL collectives never return to the host:
// a dead or stuck peer leaves every later stream synchronisation blocked
// forever.  Each communicator therefore owns a watchdog thread (the ProcessGroup
// watchdog pattern, re-done natively):
//   * every collective / p2p call enqueued outside hipGraph capture records a
//     completion event on its stream; track(stream) does the same for work the
//     communicator cannot see (a replayed hipGraph holding captured collectives);
//   * the thread polls the oldest pending event and ncclCommGetAsyncError every
//     poll interval; an event older than the timeout, or an async error, aborts
//     the communicator (ncclCommAbort makes the in-flight RCCL kernels exit, so
//     the blocked host synchronisation returns) and records the reason;
//   * every later call (and check()) raises with that reason instead of hanging.
// The thread switches itself to relaxed stream-capture mode, so its event
// queries never invalidate a capture running on the main thread.
class RcclCommunicator {
 public:
  // max_ctas > 0: at most that many channels (RCCL workgroups) per collective
  // on THIS communicator (ncclConfig_t::maxCTAs) -- the channel cap is a
  // per-communicator choice measured by the trainer (engine.py
  // select_policy), not a process-wide NCCL_MAX_NCHANNELS guess.
  RcclCommunicator(const std::string& uid, int rank, int world, int device, double timeout_s, int max_ctas = 0)
      : rank_(rank), world_(world), dev_(device), max_ctas_(max_ctas), timeout_s_(timeout_s) {
    if ((int)uid.size() != (int)sizeof(ncclUniqueId)) throw std::runtime_error("bad ncclUniqueId size");
    ncclUniqueId id;
    std::memcpy(&id, uid.data(), sizeof(id));
    DL_HIP_CHECK(hipSetDevice(device));
    ncclComm_t c = nullptr;
    if (max_ctas > 0) {
      ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
      cfg.maxCTAs = max_ctas;
      DL_NCCL_CHECK(ncclCommInitRankConfig(&c, world, id, rank, &cfg));
    } else {
      DL_NCCL_CHECK(ncclCommInitRank(&c, world, id, rank));
    }
    comm_ = Retirable<ncclComm_t>(c);
    if (timeout_s_ > 0) watcher_ = std::thread([this] { watch_loop(); });
  }
  ~RcclCommunicator() { destroy(); }

  void destroy() {
    stop_watchdog();
    ncclComm_t live = nullptr, doomed = nullptr;
    {
      std::lock_guard<std::mutex> c(call_mu_);  // no host call is in flight past this point
      std::lock_guard<std::mutex> g(mu_);
      live = comm_.take_live();
      doomed = comm_.take_doomed();
      release_events_locked();
    }
    if (live) ncclCommDestroy(live);
    if (doomed) ncclCommAbort(doomed);  // retired by the watchdog, abort still owed
  }
  // Take the communicator out of service.  With no host call in flight the
  // handle is aborted here; otherwise the last in-flight call aborts it when
  // it returns (never while RCCL may still be using it).
  void abort() {
    stop_watchdog();
    ncclComm_t c;
    {
      std::lock_guard<std::mutex> g(mu_);
      c = detach_locked("aborted by the caller");
      release_events_locked();
    }
    if (c) ncclCommAbort(c);
  }

  int rank() const { return rank_; }
  int world() const { return world_; }
  int device() const { return dev_; }
  int max_ctas() const { return max_ctas_; }

  // Every RCCL host call holds call_mu_ (RCCL calls on one communicator are not
  // thread-safe) but NOT mu_: mu_ guards only the watchdog's state (pending
  // events, abort reason), so the watchdog can always take it and mark the
  // communicator failed.  The handle itself is held through a CallGuard for
  // the duration of the call (a group: from the outermost group_start to its
  // group_end), and a failed communicator is aborted only once no call holds
  // it (retirable.h): ncclCommAbort frees the handle.
  void all_reduce(uintptr_t send, uintptr_t recv, int64_t count, int dtype, int op, uintptr_t stream) {
    std::lock_guard<std::mutex> c(call_mu_);
    CallGuard g(this);
    DL_NCCL_CHECK(ncclAllReduce((const void*)send, (void*)recv, (size_t)count, to_nccl(dtype), to_nccl_op(op),
                                g.comm, as_stream(stream)));
    enqueued(stream);
  }
  void broadcast(uintptr_t send, uintptr_t recv, int64_t count, int dtype, int root, uintptr_t stream) {
    std::lock_guard<std::mutex> c(call_mu_);
    CallGuard g(this);
    DL_NCCL_CHECK(
        ncclBroadcast((const void*)send, (void*)recv, (size_t)count, to_nccl(dtype), root, g.comm, as_stream(stream)));
    enqueued(stream);
  }
  void reduce(uintptr_t send, uintptr_t recv, int64_t count, int dtype, int op, int root, uintptr_t stream) {
    std::lock_guard<std::mutex> c(call_mu_);
    CallGuard g(this);
    DL_NCCL_CHECK(ncclReduce((const void*)send, (void*)recv, (size_t)count, to_nccl(dtype), to_nccl_op(op), root,
                             g.comm, as_stream(stream)));
    enqueued(stream);
  }
  // recvcount elements per rank
  void reduce_scatter(uintptr_t send, uintptr_t recv, int64_t recvcount, int dtype, int op, uintptr_t stream) {
    std::lock_guard<std::mutex> c(call_mu_);
    CallGuard g(this);
    DL_NCCL_CHECK(ncclReduceScatter((const void*)send, (void*)recv, (size_t)recvcount, to_nccl(dtype),
                                    to_nccl_op(op), g.comm, as_stream(stream)));
    enqueued(stream);
  }
  void all_gather(uintptr_t send, uintptr_t recv, int64_t sendcount, int dtype, uintptr_t stream) {
    std::lock_guard<std::mutex> c(call_mu_);
    CallGuard g(this);
    DL_NCCL_CHECK(
        ncclAllGather((const void*)send, (void*)recv, (size_t)sendcount, to_nccl(dtype), g.comm, as_stream(stream)));
    enqueued(stream);
  }
  void send(uintptr_t buf, int64_t count, int dtype, int peer, uintptr_t stream) {
    std::lock_guard<std::mutex> c(call_mu_);
    CallGuard g(this);
    DL_NCCL_CHECK(ncclSend((const void*)buf, (size_t)count, to_nccl(dtype), peer, g.comm, as_stream(stream)));
    enqueued(stream);
  }
  void recv(uintptr_t buf, int64_t count, int dtype, int peer, uintptr_t stream) {
    std::lock_guard<std::mutex> c(call_mu_);
    CallGuard g(this);
    DL_NCCL_CHECK(ncclRecv((void*)buf, (size_t)count, to_nccl(dtype), peer, g.comm, as_stream(stream)));
    enqueued(stream);
  }
  void group_start() {
    std::lock_guard<std::mutex> c(call_mu_);
    // the outermost group holds the handle until its group_end: RCCL issues
    // the grouped work there, with the handles the calls inside were given
    if (group_depth_ == 0) acquire_call();
    ncclResult_t r = ncclGroupStart();
    if (r != ncclSuccess) {
      if (group_depth_ == 0) release_call();
      DL_NCCL_CHECK(r);
    }
    ++group_depth_;
  }
  void group_end() {
    std::lock_guard<std::mutex> c(call_mu_);
    if (group_depth_ <= 0) throw std::runtime_error("group_end without group_start");
    ncclResult_t r = ncclGroupEnd();
    if (--group_depth_ == 0) {
      struct Release {
        RcclCommunicator* self;
        ~Release() { self->release_call(); }
      } rel{this};
      // RCCL launches grouped work (collectives AND p2p) only at the outermost
      // group end: an event recorded earlier would sit in front of the kernels
      // and complete at once, so every grouped op is timed from here
      std::vector<uintptr_t> streams;
      streams.swap(grouped_streams_);
      std::lock_guard<std::mutex> g(mu_);
      for (uintptr_t s : streams) track_locked(s);
    }
    DL_NCCL_CHECK(r);
  }
  // host calls currently holding the handle (tests)
  int inflight() {
    std::lock_guard<std::mutex> g(mu_);
    return comm_.inflight();
  }

  // pause (true) / resume the watchdog's polling, e.g. around a hipGraph
  // capture: returns only once no poll is running (pause_gate.h), so no HIP /
  // RCCL query from the watchdog thread can fall into the capture
  void set_paused(bool p) { gate_.set(mu_, p); }
  // watchdog polls run so far (tests: none may run while paused)
  long long polls() {
    std::lock_guard<std::mutex> g(mu_);
    return gate_.polls();
  }

  // Time the work enqueued so far on `stream` (no-op while it is being captured).

  void track(uintptr_t stream) {
    std::lock_guard<std::mutex> g(mu_);
    live_locked();
    track_locked(stream);
  }
  void set_timeout(double s) { timeout_s_.store(s); }
  double timeout() const { return timeout_s_.load(); }
  int pending() {
    std::lock_guard<std::mutex> g(mu_);
    return (int)pending_.size();
  }
  // "" while healthy, else why the communicator was aborted
  std::string error() {
    std::lock_guard<std::mutex> g(mu_);
    return reason_;
  }

  // Non-blocking health check: RCCL async error string, the watchdog's abort
  // reason, or "" when healthy.
  std::string async_error() {
    std::lock_guard<std::mutex> g(mu_);
    if (!reason_.empty()) return reason_;
    if (!comm_.get()) return "communicator destroyed";
    ncclResult_t r;
    DL_NCCL_CHECK(ncclCommGetAsyncError(comm_.get(), &r));
    if (r == ncclSuccess || r == ncclInProgress) return "";
    return ncclGetErrorString(r);
  }

 private:
  struct Pending {
    hipEvent_t ev;
    std::chrono::steady_clock::time_point t;
  };

  void live_locked() const {
    if (!reason_.empty()) throw std::runtime_error("RCCL communicator failed: " + reason_);
    if (!comm_.get()) throw std::runtime_error("RCCL communicator used after destroy");
  }
  // the handle for one host call if healthy (checked under mu_, used outside
  // it); every acquire_call is paired with a release_call
  ncclComm_t acquire_call() {
    std::lock_guard<std::mutex> g(mu_);
    live_locked();
    return comm_.acquire();
  }
  void release_call() {
    ncclComm_t doomed;
    {
      std::lock_guard<std::mutex> g(mu_);
      doomed = comm_.release();
    }
    if (doomed) ncclCommAbort(doomed);  // retired while this call held it
  }
  struct CallGuard {
    RcclCommunicator* self;
    ncclComm_t comm;
    explicit CallGuard(RcclCommunicator* s) : self(s), comm(s->acquire_call()) {}
    ~CallGuard() { self->release_call(); }
    CallGuard(const CallGuard&) = delete;
    CallGuard& operator=(const CallGuard&) = delete;
  };
  // after an enqueue (caller holds call_mu_): time it now, or at the outermost group end
  void enqueued(uintptr_t stream) {
    if (group_depth_ > 0) {
      grouped_streams_.push_back(stream);
      return;
    }
    std::lock_guard<std::mutex> g(mu_);
    track_locked(stream);
  }

  void track_locked(uintptr_t stream) {
    if (timeout_s_.load() <= 0 || !watcher_.joinable()) return;
    hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
    DL_HIP_CHECK(hipStreamIsCapturing(as_stream(stream), &st));
    if (st != hipStreamCaptureStatusNone) return;  // captured work is tracked at replay (track())
    hipEvent_t ev;
    if (free_.empty()) {
      DL_HIP_CHECK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    } else {
      ev = free_.back();
      free_.pop_back();
    }
    DL_HIP_CHECK(hipEventRecord(ev, as_stream(stream)));
    pending_.push_back({ev, std::chrono::steady_clock::now()});
  }

  // Record why the communicator failed and take it out of service; the caller
  // aborts the returned handle WITHOUT holding mu_ (ncclCommAbort can wait for
  // the device), so health()/error() answer immediately.  Null while a host
  // call holds the handle: that call's release_call aborts it.
  ncclComm_t detach_locked(const std::string& why) {
    if (reason_.empty()) reason_ = why;
    return comm_.retire();
  }

  void release_events_locked() {
    for (auto& p : pending_) hipEventDestroy(p.ev);
    pending_.clear();
    for (auto ev : free_) hipEventDestroy(ev);
    free_.clear();
  }

  void stop_watchdog() {
    {
      std::lock_guard<std::mutex> g(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    if (watcher_.joinable() && watcher_.get_id() != std::this_thread::get_id()) watcher_.join();
  }

  void watch_loop() {
    hipStreamCaptureMode mode = hipStreamCaptureModeRelaxed;
    (void)hipThreadExchangeStreamCaptureMode(&mode);
    (void)hipSetDevice(dev_);
    std::unique_lock<std::mutex> lk(mu_);
    while (!stop_) {
      cv_.wait_for(lk, std::chrono::milliseconds(poll_ms_));
      if (stop_) continue;
      // no HIP / RCCL query while the owner captures a hipGraph (set_paused
      // waits for a running poll to finish; pause_gate.h)
      if (!gate_.begin(lk)) continue;
      ncclComm_t dead = poll_locked();
      // dead == nullptr after a failure: a host call still holds the handle and
      // aborts it on release (release_call) -- or this loop does, after the grace
      if (dead) {  // abort outside the lock: the in-flight RCCL kernels see the abort flag and exit
        lk.unlock();
        ncclCommAbort(dead);
        lk.lock();
      }
      gate_.end(lk);
    }
  }

  // One watchdog poll (holding mu_): the handle to abort, or null.
  ncclComm_t poll_locked() {
    // A failed communicator whose handle a host call still holds is aborted by
    // that call's release -- unless the call never returns (ncclGroupEnd stuck
    // in connection setup with a dead peer, an outer group left open): after
    // the grace period the handle is aborted from here anyway, the standard
    // cross-thread abort that makes the blocked RCCL call return.
    // Its release then finds nothing left to abort.
    // Assumption: a host call still holding the handle after the
    // grace is BLOCKED inside RCCL on a peer (connection setup, proxy progress),
    // and RCCL's blocking loops poll the communicator's abort flag and return
    // ncclInternalError/ncclRemoteError without touching the communicator again
    // -- the contract NCCL documents for aborting from another thread.  A call
    // that is merely slow (not blocked) would race the free, so the grace is
    // max(5 s, the collective timeout): far longer than any RCCL host call that
    // makes progress takes (group launches and comm init: milliseconds).
    if (comm_.doomed()) {
      const auto now = std::chrono::steady_clock::now();
      if (!doomed_seen_) {
        doomed_seen_ = true;
        doomed_since_ = now;
      } else if (std::chrono::duration<double>(now - doomed_since_).count() > abort_grace_s()) {
        reason_ += " (a host call still held the communicator after the grace period: aborted from the watchdog)";
        return comm_.take_doomed();
      }
      return nullptr;
    }
    if (!comm_.get()) return nullptr;
    {
      ncclComm_t dead = nullptr;
      bool failed = false;
      // retire completed work (in order: events of one stream complete in order;
      // across streams an old unfinished event simply keeps the queue from draining)
      while (!pending_.empty()) {
        hipError_t q = hipEventQuery(pending_.front().ev);
        if (q == hipErrorNotReady) break;
        if (q != hipSuccess) {
          dead = detach_locked(std::string("HIP error while waiting for a collective: ") + hipGetErrorString(q));
          failed = true;
          break;
        }
        free_.push_back(pending_.front().ev);
        pending_.pop_front();
      }
      ncclResult_t r = ncclSuccess;
      if (!failed && ncclCommGetAsyncError(comm_.get(), &r) == ncclSuccess && r != ncclSuccess &&
          r != ncclInProgress) {
        dead = detach_locked(std::string("RCCL async error: ") + ncclGetErrorString(r));
        failed = true;
      }
      const double limit = timeout_s_.load();
      if (!failed && !pending_.empty() && limit > 0) {
        double age = std::chrono::duration<double>(std::chrono::steady_clock::now() - pending_.front().t).count();
        if (age > limit)
          dead = detach_locked("collective on rank " + std::to_string(rank_) + " did not complete within " +
                               std::to_string(limit) + " s (dead or stuck peer?)");
      }
      return dead;
    }
  }

  // seconds a doomed handle may stay held by a host call before the watchdog
  // aborts it anyway: the collective timeout, at least 5 s
  double abort_grace_s() const { return std::max(5.0, timeout_s_.load()); }

  Retirable<ncclComm_t> comm_;             // guarded by mu_
  int rank_, world_, dev_, max_ctas_;
  std::atomic<double> timeout_s_;
  int poll_ms_ = 50;
  PauseGate gate_;                          // guarded by mu_ (set() takes it)
  bool doomed_seen_ = false;                // guarded by mu_
  std::chrono::steady_clock::time_point doomed_since_;
  int group_depth_ = 0;                    // guarded by call_mu_
  std::vector<uintptr_t> grouped_streams_;  // guarded by call_mu_
  std::mutex call_mu_;                      // serialises RCCL host calls
  std::mutex mu_;                           // watchdog state: comm_, reason_, pending_, free_
  std::condition_variable cv_;
  bool stop_ = false;
  std::string reason_;
  std::deque<Pending> pending_;
  std::vector<hipEvent_t> free_;
  std::thread watcher_;
};

}  // namespace dl

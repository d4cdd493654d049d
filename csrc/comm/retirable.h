// A handle that another thread may retire (abort) while host calls use it.
//
// The communicator's watchdog must be able to take a failed RCCL communicator
// out of service at any time, but ncclCommAbort frees the handle: aborting it
// while a host call (ncclAllReduce, ncclGroupEnd, ...) is still being given or
// using the handle is a use-after-free.  So every host call holds the handle
// through acquire/release, and a retire that finds calls in flight only marks
// the handle doomed: the LAST in-flight call's release hands it back for the
// abort.  New calls fail at once (the owner checks its failure reason before
// acquire), so the in-flight count only drains.
//
// Not thread-safe by itself: every method runs under the owner's mutex, and
// the handle a method returns is aborted by the caller AFTER dropping that
// mutex (an abort may wait for the device).  Header-only and HIP-free, so the
// state machine is unit-tested on the CPU (tests/unit/test_retirable.py).
#pragma once

namespace dl {

template <class H>
class Retirable {
 public:
  Retirable() = default;
  explicit Retirable(H h) : h_(h) {}

  H get() const { return h_; }
  int inflight() const { return inflight_; }
  bool doomed() const { return doomed_ != H(); }

  // a host call starts using the handle (the caller checked it is healthy)
  H acquire() {
    ++inflight_;
    return h_;
  }
  // a host call is done; returns a doomed handle to abort now (else null)
  H release() {
    if (--inflight_ == 0 && doomed_ != H()) {
      H d = doomed_;
      doomed_ = H();
      return d;
    }
    return H();
  }
  // take the handle out of service; returns it for an immediate abort when no
  // call is in flight, else null (the last release returns it)
  H retire() {
    H c = h_;
    h_ = H();
    if (c == H()) return H();
    if (inflight_ > 0) {
      doomed_ = c;
      return H();
    }
    return c;
  }
  // destroy path: the live handle (no call can be in flight: the caller holds
  // the call lock), or a doomed one that still needs its abort
  H take_live() {
    H c = h_;
    h_ = H();
    return c;
  }
  H take_doomed() {
    H d = doomed_;
    doomed_ = H();
    return d;
  }

 private:
  H h_ = H();
  H doomed_ = H();
  int inflight_ = 0;
};

}  // namespace dl

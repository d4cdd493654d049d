// The watchdog's pause handshake.
//
// The communicator's watchdog thread polls HIP (hipEventQuery) and RCCL
// (ncclCommGetAsyncError); a HIP query from another thread while the owner
// captures a hipGraph can invalidate the capture, so captures pause the
// watchdog first (engine.py _capturing).  A bare atomic flag is not a pause:
// a poll that had already passed its check before the flag was set still ran
// its queries during the capture.  Here every poll is
// bracketed by begin()/end() under the owner's mutex, and set(true) takes the
// same mutex and waits until no poll is running -- including the part of a
// poll run WITHOUT the mutex (the watchdog drops it around ncclCommAbort) --
// so once set(true) returns no poll is in progress and none starts until
// set(false).
//
// Header-only and HIP-free: the handshake is unit-tested on the CPU under
// ThreadSanitizer (tests/unit/native/pause_gate_test.cpp).
#pragma once
#include <condition_variable>
#include <mutex>

namespace dl {

class PauseGate {
 public:
  // Watchdog, holding `lk` on the owner's mutex: whether a poll may start
  // now (not paused); if so the poll is marked running until end().
  bool begin(std::unique_lock<std::mutex>& lk) {
    (void)lk;
    if (paused_) return false;
    busy_ = true;
    ++polls_;
    return true;
  }
  // Watchdog, holding `lk` again: the poll begun last is over.
  void end(std::unique_lock<std::mutex>& lk) {
    (void)lk;
    busy_ = false;
    idle_.notify_all();
  }
  // Owner thread (must not hold `mu`): pause -- returns once no poll is
  // running -- or resume.
  void set(std::mutex& mu, bool paused) {
    std::unique_lock<std::mutex> lk(mu);
    paused_ = paused;
    if (paused) idle_.wait(lk, [this] { return !busy_; });
  }
  // (holding the owner's mutex) state for tests / diagnostics
  bool paused() const { return paused_; }
  bool busy() const { return busy_; }
  long long polls() const { return polls_; }

 private:
  bool paused_ = false;
  bool busy_ = false;
  long long polls_ = 0;
  std::condition_variable idle_;
};

}  // namespace dl

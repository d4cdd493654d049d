// CPU test of the communicator's handle-retirement state machine
// (csrc/comm/retirable.h): a watchdog that fails the communicator while a
// host call is inside RCCL must not abort (free) the handle until that call
// has returned.  The "handle" is an int id; "abort" checks that no call is
// using it.  Built and run by tests/unit/test_retirable.py with g++ -pthread.
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <mutex>
#include <random>
#include <thread>
#include <vector>

#include "comm/retirable.h"

using dl::Retirable;

static int fails = 0;
#define CHECK(c)                                                 \
  do {                                                           \
    if (!(c)) {                                                  \
      std::fprintf(stderr, "CHECK failed: %s (line %d)\n", #c, __LINE__); \
      ++fails;                                                   \
    }                                                            \
  } while (0)

static void state_machine() {
  // idle retire: aborted at once
  Retirable<int> a(7);
  CHECK(a.retire() == 7);
  CHECK(a.get() == 0 && !a.doomed());
  CHECK(a.retire() == 0);  // second retire: nothing left
  // retire while one call is in flight: deferred to its release
  Retirable<int> b(9);
  CHECK(b.acquire() == 9);
  CHECK(b.retire() == 0);
  CHECK(b.doomed() && b.get() == 0);
  CHECK(b.release() == 9);
  CHECK(!b.doomed() && b.inflight() == 0);
  // nested holders (a group + a call inside it): only the last release aborts
  Retirable<int> c(5);
  c.acquire();
  c.acquire();
  CHECK(c.retire() == 0);
  CHECK(c.release() == 0);
  CHECK(c.release() == 5);
  // healthy release returns nothing
  Retirable<int> d(3);
  d.acquire();
  CHECK(d.release() == 0 && d.get() == 3);
  // a call that never returns: after the grace period the watchdog takes the
  // doomed handle and aborts it anyway; the late release finds nothing to abort
  Retirable<int> f(6);
  f.acquire();
  CHECK(f.retire() == 0 && f.doomed());
  CHECK(f.take_doomed() == 6);
  CHECK(f.release() == 0 && !f.doomed() && f.inflight() == 0);
  // destroy path
  Retirable<int> e(4);
  e.acquire();
  e.retire();
  CHECK(e.take_live() == 0);
  CHECK(e.take_doomed() == 4);
}

// Threads: K callers repeatedly acquire the handle (under the owner's mutex,
// failing once it is retired), "use" it outside the mutex, then release; a
// watchdog retires it at a random moment.  Abort must run exactly once and
// only when no caller is using the handle.
static void threaded(unsigned seed) {
  std::mutex mu;
  Retirable<int> h(42);
  bool failed = false;
  std::atomic<int> using_now{0};
  std::atomic<int> aborts{0};
  std::atomic<bool> bad_abort{false};
  auto do_abort = [&](int handle) {
    if (handle != 42 || using_now.load() != 0) bad_abort = true;
    aborts.fetch_add(1);
  };
  std::mt19937 rng(seed);
  const int delay_us = (int)(rng() % 2000);
  std::vector<std::thread> callers;
  for (int k = 0; k < 4; ++k) {
    callers.emplace_back([&, k] {
      std::mt19937 r(seed * 31 + k);
      for (int it = 0; it < 200; ++it) {
        int handle;
        {
          std::lock_guard<std::mutex> g(mu);
          if (failed) return;  // live_locked() throws: no new call
          handle = h.acquire();
        }
        using_now.fetch_add(1);
        if (handle != 42) bad_abort = true;
        std::this_thread::sleep_for(std::chrono::microseconds(r() % 50));  // "inside RCCL"
        using_now.fetch_sub(1);
        int doomed;
        {
          std::lock_guard<std::mutex> g(mu);
          doomed = h.release();
        }
        if (doomed) do_abort(doomed);
      }
    });
  }
  std::thread watchdog([&] {
    std::this_thread::sleep_for(std::chrono::microseconds(delay_us));
    int dead;
    {
      std::lock_guard<std::mutex> g(mu);
      failed = true;
      dead = h.retire();
    }
    if (dead) do_abort(dead);
  });
  for (auto& t : callers) t.join();
  watchdog.join();
  CHECK(!bad_abort.load());
  CHECK(aborts.load() == 1);
  CHECK(h.inflight() == 0 && !h.doomed() && h.get() == 0);
}

int main() {
  state_machine();
  for (unsigned s = 1; s <= 200; ++s) threaded(s);
  if (fails) {
    std::fprintf(stderr, "%d failures\n", fails);
    return 1;
  }
  std::printf("retirable: ok\n");
  return 0;
}

// CPU test of the watchdog's pause handshake (csrc/comm/pause_gate.h): once
// set(true) returns, no poll is running -- including a poll that was already
// past its pause check, and the part of a poll run without the owner's mutex
// (the communicator drops it around ncclCommAbort) -- and none starts until
// set(false).  The watchdog here is the communicator's loop shape with the
// HIP / RCCL queries replaced by sleeps that flag "a query is running".
// Built and run under ThreadSanitizer by tests/unit/test_capture_guard.py.
#include <atomic>
#include <chrono>
#include <cstdio>
#include <mutex>
#include <random>
#include <thread>

#include "comm/pause_gate.h"

static int fails = 0;
#define CHECK(c)                                                          \
  do {                                                                    \
    if (!(c)) {                                                           \
      std::fprintf(stderr, "CHECK failed: %s (line %d)\n", #c, __LINE__); \
      ++fails;                                                            \
    }                                                                     \
  } while (0)

int main() {
  std::mutex mu;
  dl::PauseGate gate;
  bool stop = false;
  std::atomic<int> querying{0};      // > 0 while a "HIP query" of a poll runs
  std::atomic<long long> queries{0};  // completed queries
  std::thread watchdog([&] {
    std::mt19937 r(7);
    std::unique_lock<std::mutex> lk(mu);
    while (!stop) {
      // (the communicator waits on a condition variable with a timeout here;
      // libtsan of this g++ does not intercept pthread_cond_clockwait, so the
      // driver sleeps unlocked instead)
      lk.unlock();
      std::this_thread::sleep_for(std::chrono::microseconds(50));
      lk.lock();
      if (stop) continue;
      if (!gate.begin(lk)) continue;
      // the locked part of the poll (hipEventQuery / ncclCommGetAsyncError)
      querying.fetch_add(1);
      std::this_thread::sleep_for(std::chrono::microseconds(r() % 200));
      querying.fetch_sub(1);
      queries.fetch_add(1);
      if (r() % 4 == 0) {  // the unlocked part (ncclCommAbort outside mu)
        lk.unlock();
        querying.fetch_add(1);
        std::this_thread::sleep_for(std::chrono::microseconds(r() % 200));
        querying.fetch_sub(1);
        lk.lock();
      }
      gate.end(lk);
    }
  });
  std::mt19937 r(11);
  long long paused_polls = 0;
  for (int it = 0; it < 400; ++it) {
    std::this_thread::sleep_for(std::chrono::microseconds(r() % 300));  // the watchdog runs freely
    gate.set(mu, true);                                                 // capture begins
    CHECK(querying.load() == 0);
    const long long before = queries.load();
    {
      std::lock_guard<std::mutex> g(mu);
      CHECK(gate.paused() && !gate.busy());
      paused_polls = gate.polls();
    }
    std::this_thread::sleep_for(std::chrono::microseconds(200 + r() % 300));  // "the capture"
    CHECK(querying.load() == 0);
    CHECK(queries.load() == before);
    {
      std::lock_guard<std::mutex> g(mu);
      CHECK(gate.polls() == paused_polls);
    }
    gate.set(mu, false);  // capture ended
  }
  {
    std::lock_guard<std::mutex> g(mu);
    stop = true;
  }
  watchdog.join();
  CHECK(queries.load() > 0);
  if (fails) {
    std::fprintf(stderr, "%d failures\n", fails);
    return 1;
  }
  std::printf("pause_gate: ok (%lld polls)\n", queries.load());
  return 0;
}

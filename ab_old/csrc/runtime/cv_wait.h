// Condition-variable timed waits for the runtime.  Normal builds wait on the
// steady clock.  ThreadSanitizer builds (-DDTF_TSAN, scripts/asan_runtime.py
// --tsan) wait on the system clock instead: libstdc++ implements steady-clock
// waits with pthread_cond_clockwait, which GCC 11's libtsan does not intercept,
// so TSan would miss the wait's unlock/relock and report the queue's own
// mutex-protected accesses as races.
#pragma once
#include <chrono>
#include <condition_variable>
#include <mutex>

namespace dtf {

template <class Pred>
bool cv_wait_until(std::condition_variable& cv, std::unique_lock<std::mutex>& lk,
                   std::chrono::steady_clock::time_point deadline, Pred pred) {
#ifdef DTF_TSAN
  const auto sys = std::chrono::system_clock::now() +
                   std::chrono::duration_cast<std::chrono::system_clock::duration>(deadline - std::chrono::steady_clock::now());
  return cv.wait_until(lk, sys, pred);
#else
  return cv.wait_until(lk, deadline, pred);
#endif
}

template <class Rep, class Period, class Pred>
bool cv_wait_for(std::condition_variable& cv, std::unique_lock<std::mutex>& lk,
                 std::chrono::duration<Rep, Period> d, Pred pred) {
  return cv_wait_until(cv, lk,
                       std::chrono::steady_clock::now() + std::chrono::duration_cast<std::chrono::steady_clock::duration>(d),
                       pred);
}

}  // namespace dtf

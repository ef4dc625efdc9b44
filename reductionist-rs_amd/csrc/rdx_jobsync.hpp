// The coalescer's hand-off of one request between its caller and the dispatcher that completes it
// (rdx_runtime.cpp Job): one atomic word, so that the completing side's last access to the caller's
// (stack-allocated) job is the exchange that publishes the result.  Host code; tested under
// ThreadSanitizer by tests/test_sanitize_cpu.py (tests/cpp/test_jobsync.cpp).
#pragma once
#include <linux/futex.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <atomic>
#include <cstdint>
#include <ctime>

namespace rdx {

// state: kJobPending -> (the caller gives up spinning) kJobSleeping -> kJobDone
constexpr uint32_t kJobPending = 0, kJobSleeping = 1, kJobDone = 2;

// Completion: the caller's outputs are written; release them and wake the caller only if it sleeps.  The
// exchange both publishes the result and tells whether the caller went to sleep, and it is the last access
// to the job (the futex wake-up names the address; it reads no memory there).
inline void job_finish(std::atomic<uint32_t> &state) {
    uint32_t *const word = reinterpret_cast<uint32_t *>(&state);
    if (state.exchange(kJobDone, std::memory_order_acq_rel) == kJobSleeping)
        syscall(SYS_futex, word, FUTEX_WAKE_PRIVATE, 1, nullptr, nullptr, 0);
}

// The caller's wait: spin `spin` pause iterations (a result arrives within tens of microseconds of its
// launch), then announce the sleep with a CAS pending -> sleeping and sleep on the futex, re-checking every
// millisecond.  A failed CAS means the job is done.
inline void job_wait(std::atomic<uint32_t> &state, int spin) {
    for (int i = 0; i < spin; ++i) {
        if (state.load(std::memory_order_acquire) == kJobDone) return;
        __builtin_ia32_pause();
    }
    uint32_t expect = kJobPending;
    if (!state.compare_exchange_strong(expect, kJobSleeping, std::memory_order_acq_rel)) return;
    while (state.load(std::memory_order_acquire) != kJobDone) {
        const timespec ts{0, 1000000};
        syscall(SYS_futex, reinterpret_cast<uint32_t *>(&state), FUTEX_WAIT_PRIVATE, kJobSleeping, &ts, nullptr, 0);
    }
}

}  // namespace rdx

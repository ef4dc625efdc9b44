// The coalescer's job hand-off (reductionist-rs_amd/csrc/rdx_jobsync.hpp) under ThreadSanitizer: many
// short-lived callers, each with its job on its own stack (as execute_host's resident path and the direct
// runner do), queued to one dispatcher thread that writes the result and completes the job.  Callers spin
// 0, 1 or 200 iterations before sleeping, so every interleaving of finish and the pending -> sleeping CAS
// occurs.  A use of the job after its caller returned, or an unsynchronised result, is a TSan report.
#include <atomic>
#include <cstdio>
#include <deque>
#include <mutex>
#include <thread>
#include <vector>

#include "../../reductionist-rs_amd/csrc/rdx_jobsync.hpp"

struct Job {
    uint64_t payload = 0, result = 0;
    std::atomic<uint32_t> state{rdx::kJobPending};
};

int main(int argc, char **argv) {
    const int callers = argc > 1 ? std::atoi(argv[1]) : 8, per = argc > 2 ? std::atoi(argv[2]) : 2000;
    std::mutex mu;
    std::deque<Job *> q;
    std::atomic<bool> stop{false};
    std::atomic<long> bad{0};
    std::thread dispatcher([&] {
        std::vector<Job *> batch;
        while (!stop.load(std::memory_order_acquire)) {
            {
                std::lock_guard<std::mutex> g(mu);
                while (!q.empty() && batch.size() < 5) {
                    batch.push_back(q.front());
                    q.pop_front();
                }
            }
            for (Job *j : batch) {
                j->result = j->payload * 3 + 1;   // the outputs, then the exchange: the last access
                rdx::job_finish(j->state);
            }
            if (batch.empty()) std::this_thread::yield();
            batch.clear();
        }
    });
    std::vector<std::thread> th;
    for (int c = 0; c < callers; ++c)
        th.emplace_back([&, c] {
            const int spins[3] = {0, 1, 200};
            for (int i = 0; i < per; ++i) {
                Job j;   // on this caller's stack, reused by the next iteration
                j.payload = (uint64_t)c << 32 | (uint64_t)i;
                {
                    std::lock_guard<std::mutex> g(mu);
                    q.push_back(&j);
                }
                rdx::job_wait(j.state, spins[(c + i) % 3]);
                if (j.result != j.payload * 3 + 1) ++bad;
            }
        });
    for (auto &t : th) t.join();
    stop.store(true, std::memory_order_release);
    dispatcher.join();
    if (bad.load()) {
        std::printf("jobsync: %ld wrong results\n", bad.load());
        return 1;
    }
    std::printf("jobsync: ok (%d callers x %d jobs)\n", callers, per);
    return 0;
}

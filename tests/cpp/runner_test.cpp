// The host-ingest coordinator threads (aws-crt-cpp_amd/csrc/runner.h), under TSan: tasks posted
// close together run concurrently.  Task A waits for a flag only task B sets; on one shared thread A
// would wait out its timeout (two posts both saw one idle thread and ran one after the
// other).  Built and run by tests/test_host_ingest.py.
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <memory>
#include <mutex>
#include <thread>

#include "runner.h"

namespace {
int fails = 0;
#define CHECK(c)                                                              \
    do {                                                                      \
        if (!(c)) {                                                           \
            std::printf("FAIL %s:%d %s\n", __FILE__, __LINE__, #c);          \
            ++fails;                                                          \
        }                                                                     \
    } while (0)

struct Latch {
    std::mutex mu;
    std::condition_variable cv;
    int n = 0;
    void arrive() {
        std::lock_guard<std::mutex> g(mu);
        ++n;
        cv.notify_all();
    }
    bool wait_for(int k, int ms) {
        std::unique_lock<std::mutex> g(mu);
        // system_clock: libstdc++ waits on it with pthread_cond_timedwait, which TSan intercepts (the
        // steady_clock wait goes through pthread_cond_clockwait, which gcc 11's TSan does not see)
        return cv.wait_until(g, std::chrono::system_clock::now() + std::chrono::milliseconds(ms), [&] { return n >= k; });
    }
};

// k tasks that each wait for all k to have started: they complete only if they run at once
// (the latches are shared with the tasks: a task that timed out may still be running when the round
// returns)
struct Round {
    Latch started, done;
    std::atomic<int> ok{0};
};
bool round_concurrent(amdcrc::Runner &r, int k, int wait_ms = 10000) {
    auto R = std::make_shared<Round>();
    for (int i = 0; i < k; ++i)
        r.post([R, k, wait_ms] {
            R->started.arrive();
            if (R->started.wait_for(k, wait_ms)) R->ok.fetch_add(1);
            R->done.arrive();
        });
    R->done.wait_for(k, 30000);
    return R->ok.load() == k;
}
}  // namespace

int main() {
    {
        amdcrc::Runner r;
        // warm: one idle thread exists before the pair is posted (the round-4 failure case)
        CHECK(round_concurrent(r, 1));
        std::this_thread::sleep_for(std::chrono::milliseconds(20));
        CHECK(round_concurrent(r, 2));
        // the pair again and again, every thread idle before it (the race is a matter of timing)
        int bad = 0;
        for (int i = 0; i < 100 && bad == 0; ++i) {
            std::this_thread::sleep_for(std::chrono::milliseconds(2));
            bad += !round_concurrent(r, 2, 2000);
        }
        CHECK(bad == 0);
        // the invariant behind it, independent of timing: once the posts of a pair have returned, the
        // pair has two threads (the one idle thread and a new one), whoever wins the wake-up race
        for (int i = 0; i < 20; ++i) {
            amdcrc::Runner fresh;
            CHECK(round_concurrent(fresh, 1));  // one thread, idle after this
            std::this_thread::sleep_for(std::chrono::milliseconds(2));
            auto G = std::make_shared<Round>();
            for (int j = 0; j < 2; ++j)
                fresh.post([G] {
                    G->started.wait_for(1, 10000);  // the gate
                    G->done.arrive();
                });
            const size_t after = fresh.threads();
            G->started.arrive();
            G->done.wait_for(2, 30000);
            CHECK(after >= 2);  // (3 if the first thread was not idle yet)
        }
        // posts from two threads at once
        auto R = std::make_shared<Round>();
        auto job = [R] {
            R->started.arrive();
            if (R->started.wait_for(2, 10000)) R->ok.fetch_add(1);
            R->done.arrive();
        };
        std::thread a([&] { r.post(job); }), b([&] { r.post(job); });
        a.join();
        b.join();
        R->done.wait_for(2, 30000);
        CHECK(R->ok.load() == 2);
        // eight at once, then threads are reused: a later pair starts no new thread
        CHECK(round_concurrent(r, 8));
        std::this_thread::sleep_for(std::chrono::milliseconds(20));
        const size_t t = r.threads();
        CHECK(round_concurrent(r, 2));
        std::this_thread::sleep_for(std::chrono::milliseconds(20));
        CHECK(r.threads() == t);
        CHECK(t <= 12);
    }
    std::printf(fails ? "[FAIL] RunnerConcurrent\n" : "[PASS] RunnerConcurrent\n");
    return fails ? 1 : 0;
}

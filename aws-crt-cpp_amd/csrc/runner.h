// Threads that run host-ingest jobs' coordinators (ingest.cpp), kept for reuse: a std::thread per job
// cost its creation, ~0.1 ms, on every job.  Every queued task has a thread of its own -- one is
// started whenever the queued tasks outnumber the idle threads -- so concurrent jobs run concurrently.
// (Round 4 started a thread only when no thread was idle; an idle thread counts itself busy only once
// it runs, so two posts close together both found one idle thread and their jobs ran one after the
// other on it.)  Header-only so tests/cpp/runner_test.cpp can check that under TSan.
#pragma once

#include <condition_variable>
#include <deque>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace amdcrc {

class Runner {
  public:
    void post(std::function<void()> f) {
        std::lock_guard<std::mutex> g(mu_);
        q_.push_back(std::move(f));
        if (q_.size() > idle_) ts_.emplace_back([this] { loop(); });
        cv_.notify_one();
    }
    ~Runner() {
        {
            std::lock_guard<std::mutex> g(mu_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto &t : ts_) t.join();
    }
    size_t threads() {
        std::lock_guard<std::mutex> g(mu_);
        return ts_.size();
    }

  private:
    void loop() {
        std::unique_lock<std::mutex> g(mu_);
        for (;;) {
            ++idle_;
            cv_.wait(g, [this] { return stop_ || !q_.empty(); });
            --idle_;
            if (q_.empty()) return;  // stopping
            std::function<void()> f = std::move(q_.front());
            q_.pop_front();
            g.unlock();
            f();
            g.lock();
        }
    }
    std::mutex mu_;
    std::condition_variable cv_;
    std::deque<std::function<void()>> q_;
    std::vector<std::thread> ts_;
    size_t idle_ = 0;  // threads waiting for a task (a woken thread leaves the count when it runs)
    bool stop_ = false;
};

}  // namespace amdcrc

// Per-stream engine state with a bounded lifetime (round 4).
//
// Kernels on one stream are serialised, so the engine gives every stream it launches on its own
// scratch (cross-tile workspace, descriptor staging, XXH3 block sums, multipart results): launches on
// different streams never share it.  Round 3 kept that state in maps keyed by stream handle that were
// never pruned, so a service that creates a stream per request grew device and pinned memory without
// bound.  StreamStates keeps at most `max_live` entries: a new stream beyond that takes over the state
// of the least recently used stream whose work on it has completed (its fence), and a released stream
// (aws_crt_amd_stream_release) hands its state back at once.  Handed-back states are reused, never
// freed (freeing device memory may synchronise the device), so the memory held is bounded by the
// largest number of streams whose engine work was in flight at one time plus max_live.
//
// Header-only and HIP-free: the policy P supplies `static bool idle(const State &)` (no queued launch
// reads the state: its fence event has completed, it is not referenced by a captured graph, no call
// holds it).  tests/cpp/stream_states_test.cpp drives it with host stand-ins.
#pragma once

#include <cstddef>
#include <cstdint>
#include <memory>
#include <unordered_map>
#include <vector>

namespace amdcrc {

template <class Key, class State, class P>
class StreamStates {
   public:
    explicit StreamStates(size_t max_live) : max_live_(max_live ? max_live : 1) {}

    // The state of stream s, creating or adopting one; *fresh tells a caller that the entry was not
    // this stream's before (its memory may still be sized for another stream's work).
    State *get(const Key &s, bool *fresh = nullptr) {
        ++tick_;
        auto it = live_.find(s);
        if (it != live_.end()) {
            it->second->tick = tick_;
            if (fresh) *fresh = false;
            return it->second.get();
        }
        if (fresh) *fresh = true;
        if (live_.size() >= max_live_) evict_lru();
        std::unique_ptr<State> st;
        for (size_t i = 0; i < spare_.size(); ++i)
            if (P::idle(*spare_[i])) {
                st = std::move(spare_[i]);
                spare_.erase(spare_.begin() + (long)i);
                break;
            }
        if (!st) {
            st.reset(new State());
            ++created_;
        }
        st->tick = tick_;
        State *raw = st.get();
        live_.emplace(s, std::move(st));
        return raw;
    }

    // Stream s will not be used again (or not soon): its state goes back to the spares.  Safe while
    // its last launches still run -- a spare is reused only once idle.
    bool release(const Key &s) {
        auto it = live_.find(s);
        if (it == live_.end()) return false;
        spare_.push_back(std::move(it->second));
        live_.erase(it);
        return true;
    }

    size_t live() const { return live_.size(); }
    size_t spares() const { return spare_.size(); }
    size_t created() const { return created_; }  // states ever allocated: the memory bound

    template <class F>
    void for_each(F &&f) {
        for (auto &kv : live_) f(*kv.second);
        for (auto &sp : spare_) f(*sp);
    }

   private:
    // the least recently used idle entries go to the spares until there is room (busy ones stay)
    void evict_lru() {
        while (live_.size() >= max_live_) {
            auto best = live_.end();
            for (auto it = live_.begin(); it != live_.end(); ++it)
                if (P::idle(*it->second) && (best == live_.end() || it->second->tick < best->second->tick)) best = it;
            if (best == live_.end()) return;  // every live stream has work in flight: grow instead
            spare_.push_back(std::move(best->second));
            live_.erase(best);
        }
    }

    size_t max_live_;
    uint64_t tick_ = 0;
    size_t created_ = 0;
    std::unordered_map<Key, std::unique_ptr<State>> live_;
    std::vector<std::unique_ptr<State>> spare_;
};

}  // namespace amdcrc

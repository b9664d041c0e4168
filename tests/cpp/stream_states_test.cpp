// CPU model of the engine's per-stream state lifetime (aws-crt-cpp_amd/csrc/stream_states.h), built
// under ASan + UBSan by tests/test_stream_states.py.  Host stand-ins: a "stream" is an integer handle
// (recycled like the HIP runtime recycles stream objects), a state's "device memory" is a host
// allocation, and its fence completes when the test says the stream's work has finished.
#include <cassert>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "stream_states.h"

namespace {
size_t g_bytes = 0;  // "device" bytes held by all states
struct State {
    std::vector<unsigned char> scratch;  // grows on first use, like the workspace / staging
    bool busy = false;                   // a launch that reads it is in flight
    uint64_t tick = 0;
    State() {
        scratch.resize(1 << 16);
        g_bytes += scratch.size();
    }
    ~State() { g_bytes -= scratch.size(); }
};
struct Policy {
    static bool idle(State &s) { return !s.busy; }
};
using Cache = amdcrc::StreamStates<int, State, Policy>;

int fails = 0;
#define CHECK(c)                                                              \
    do {                                                                      \
        if (!(c)) {                                                           \
            std::printf("FAIL %s:%d %s\n", __FILE__, __LINE__, #c);            \
            ++fails;                                                          \
        }                                                                     \
    } while (0)

// 1,000 streams created, used once and destroyed, some released, some not: states stay bounded
void thousand_streams_sequential() {
    Cache c(64);
    for (int i = 0; i < 1000; ++i) {
        const int handle = 1000 + i;  // every stream a new handle
        State *s = c.get(handle);
        s->busy = true;   // a launch reads it
        s->busy = false;  // ... and has completed
        if (i % 3 == 0) c.release(handle);
    }
    CHECK(c.created() <= 65);
    CHECK(c.live() <= 64);
    CHECK(g_bytes <= 65u * (1u << 16));
    std::printf("sequential: created %zu live %zu spare %zu\n", c.created(), c.live(), c.spares());
}

// a stream whose work is in flight keeps its state; the LRU idle one is taken over instead
void busy_states_are_kept() {
    Cache c(4);
    State *a = c.get(1);
    a->busy = true;
    State *b = c.get(2);
    c.get(3);
    c.get(4);
    State *e = c.get(5);  // evicts the LRU idle one (2), not the busy 1
    CHECK(e == b);
    CHECK(c.get(1) == a);
    // every live stream busy: the cache grows past its bound rather than hand over a busy state
    Cache d(2);
    State *x = d.get(10), *y = d.get(11);
    x->busy = y->busy = true;
    State *z = d.get(12);
    CHECK(z != x && z != y && d.created() == 3);
    x->busy = y->busy = false;
}

// a released state is reused only once idle; a recycled handle gets a fresh entry after release
void release_and_recycled_handles() {
    Cache c(8);
    State *s = c.get(7);
    s->busy = true;
    c.release(7);           // released with its launch still in flight
    State *t = c.get(7);    // the same handle again (a new stream at the same address)
    CHECK(t != s);          // not the busy one
    s->busy = false;
    c.release(7);
    State *u = c.get(8);    // now a spare is idle: reused, nothing new allocated
    CHECK(u == s || u == t);
    CHECK(c.created() == 2);
}

// concurrency of streams: K streams in flight at once, 1,000 streams in total
void interleaved_in_flight() {
    Cache c(64);
    const int K = 16;
    std::vector<std::pair<int, State *>> inflight;
    for (int i = 0; i < 1000; ++i) {
        State *s = c.get(5000 + i);
        s->busy = true;
        inflight.push_back({5000 + i, s});
        if ((int)inflight.size() > K) {  // the oldest stream finishes and is destroyed
            inflight.front().second->busy = false;
            if (i % 2) c.release(inflight.front().first);
            inflight.erase(inflight.begin());
        }
    }
    for (auto &p : inflight) p.second->busy = false;
    CHECK(c.created() <= 64 + K + 1);
    std::printf("interleaved: created %zu live %zu spare %zu\n", c.created(), c.live(), c.spares());
}
}  // namespace

int main() {
    thousand_streams_sequential();
    busy_states_are_kept();
    release_and_recycled_handles();
    interleaved_in_flight();
    CHECK(g_bytes == 0);  // every state freed with its cache
    if (fails) return 1;
    std::printf("[PASS] StreamStatesBounded\n");
    return 0;
}

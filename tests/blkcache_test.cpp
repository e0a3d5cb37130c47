// CPU test of the process-memory lifetime rules (mimic_amd/csrc/blkcache.h, used by engine.cpp's
// NewProcess / Run / Cleanup).  A fake device runs queued work items on a thread of its own, in
// order, like one HIP stream; fences mark a queue position.  Many threads create, use and clean up
// "processes" at once (processPool's workers and Handoff goroutines, vm.go:548-573).  Checked:
//  * a block handed out by the cache has no pending work of an earlier owner (take waits for the
//    fence of the block's last use);
//  * while any work item runs on a block, no other process holds that block;
//  * a block released after a sync that covered its last enqueue needs no fence (SeqClock);
//  * the cache refuses blocks beyond its cap.
// Built and run by tests/test_blkcache.py (g++, ThreadSanitizer when available).
#include <assert.h>
#include <stdio.h>
#include <stdlib.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <functional>
#include <mutex>
#include <random>
#include <thread>
#include <unordered_map>

#include "../mimic_amd/csrc/blkcache.h"

static std::atomic<int> failures{0};
#define CHECK(c, ...)                                  \
    do {                                               \
        if (!(c)) {                                    \
            fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
            fprintf(stderr, __VA_ARGS__);              \
            fprintf(stderr, "\n");                     \
            failures++;                                \
        }                                              \
    } while (0)

// one in-order queue (the VM's stream)
struct FakeStream {
    std::mutex mu;
    std::condition_variable cv, done_cv;
    std::deque<std::pair<uint64_t, std::function<void()>>> q;
    uint64_t submitted = 0, completed = 0;
    bool stop = false;
    std::thread worker;
    FakeStream() {
        worker = std::thread([this] {
            for (;;) {
                std::pair<uint64_t, std::function<void()>> it;
                {
                    std::unique_lock<std::mutex> lk(mu);
                    cv.wait(lk, [this] { return stop || !q.empty(); });
                    if (q.empty()) return;
                    it = std::move(q.front());
                    q.pop_front();
                }
                it.second();
                {
                    std::lock_guard<std::mutex> lk(mu);
                    completed = it.first;
                }
                done_cv.notify_all();
            }
        });
    }
    ~FakeStream() {
        {
            std::lock_guard<std::mutex> lk(mu);
            stop = true;
        }
        cv.notify_all();
        worker.join();
    }
    uint64_t enqueue(std::function<void()> f) {
        uint64_t n;
        {
            std::lock_guard<std::mutex> lk(mu);
            n = ++submitted;
            q.emplace_back(n, std::move(f));
        }
        cv.notify_all();
        return n;
    }
    uint64_t tail() {
        std::lock_guard<std::mutex> lk(mu);
        return submitted;
    }
    void wait_for(uint64_t n) {
        std::unique_lock<std::mutex> lk(mu);
        done_cv.wait(lk, [&] { return completed >= n; });
    }
    bool passed(uint64_t n) {
        std::lock_guard<std::mutex> lk(mu);
        return completed >= n;
    }
};

struct FakeFence : BlkFence {
    FakeStream *s;
    uint64_t at;
    FakeFence(FakeStream *s_, uint64_t at_) : s(s_), at(at_) {}
    void wait() override { s->wait_for(at); }
};

// per fake block: the process holding it and the work items queued on it
struct BlockState {
    std::atomic<int> holder{0};
    std::atomic<int> pending{0};
};
static std::mutex states_mu;
static std::unordered_map<uint8_t *, BlockState *> states;
static BlockState *state_of(uint8_t *p) {
    std::lock_guard<std::mutex> lk(states_mu);
    auto &s = states[p];
    if (!s) s = new BlockState();
    return s;
}

static void test_fence_wait() {
    FakeStream st;
    BlkCache cache(1 << 20);
    static uint8_t mem[2048];
    Blk b;
    b.dev = mem;
    b.cls = BlkCache::size_class(1500);
    std::atomic<int> word{0};
    // process 1's work on the block, still running when it is cleaned up
    const uint64_t n = st.enqueue([&] {
        std::this_thread::sleep_for(std::chrono::milliseconds(50));
        word = 1;
    });
    CHECK(cache.give(b, std::make_shared<FakeFence>(&st, n)), "give refused");
    Blk c;
    CHECK(cache.take(1200, false, &c), "take found nothing");
    CHECK(c.dev == mem, "a different block");
    CHECK(st.passed(n), "take returned before the fence of the block's last use");
    CHECK(word.load() == 1, "the old work had not finished when the block was handed out");
    CHECK(!c.fence, "the fence stays with the block");
    Blk d;
    CHECK(!cache.take(1200, false, &d), "one block handed out twice");
    CHECK(!cache.take(1200, true, &d), "a device-only block handed out as one with a host half");
}

static void test_cap() {
    BlkCache cache(4096);
    static uint8_t m1[2048], m2[2048], m3[2048], h3[2048];
    Blk a, b, c;
    a.dev = m1;
    a.cls = 2048;
    b.dev = m2;
    b.cls = 2048;
    c.dev = m3;
    c.host = h3;
    c.cls = 2048;
    CHECK(cache.give(a, nullptr) && cache.give(b, nullptr), "refused under the cap");
    CHECK(!cache.give(c, nullptr), "kept past the cap");
    CHECK(cache.cached_bytes() == 4096, "cached %zu", cache.cached_bytes());
    Blk x;
    CHECK(cache.take(2000, false, &x) && cache.cached_bytes() == 2048, "take did not release the bytes");
    CHECK(BlkCache::size_class(1) == 1024 && BlkCache::size_class(1025) == 2048 && BlkCache::size_class(4096) == 4096,
          "size classes");
}

static void test_seqclock() {
    SeqClock c;
    const uint64_t a = c.next(), b = c.next();
    CHECK(!c.idle(a) && !c.idle(b), "idle before any sync");
    c.complete(a);
    CHECK(c.idle(a) && !c.idle(b), "complete(a) covers a only");
    c.complete(b);
    c.complete(a);   // an older sync finishing late must not move `done` back
    CHECK(c.idle(b), "done moved back");
    CHECK(c.idle(0), "a process that never enqueued is idle");
}

// the engine's pattern from many threads: NewProcess (take or allocate, upload), Run (launch +
// sync), sometimes Cleanup right after NewProcess with the upload still queued, Cleanup on another
// thread (Handoff)
static void test_threads() {
    FakeStream st;
    BlkCache cache(64 << 10);   // small: blocks are also freed past the cap
    SeqClock seq;
    std::recursive_mutex run_mu;
    std::atomic<int> allocs{0}, frees{0};
    auto work_on = [&](uint8_t *blk, int pid) {   // run_mu held
        BlockState *s = state_of(blk);
        s->pending++;
        const uint64_t n = st.enqueue([s, pid] {
            const int h = s->holder.load();
            CHECK(h == pid || h == 0, "work of process %d ran while process %d held its block", pid, h);
            std::this_thread::sleep_for(std::chrono::microseconds(20));
            s->pending--;
        });
        (void)n;
        return seq.next();
    };
    auto sync = [&]() {   // run_mu held
        const uint64_t upto = seq.issued();
        st.wait_for(st.tail());
        seq.complete(upto);
    };
    auto release = [&](Blk &b, uint64_t last) {
        std::shared_ptr<BlkFence> f;
        if (!seq.idle(last)) f = std::make_shared<FakeFence>(&st, st.tail());
        state_of(b.dev)->holder = 0;
        if (!cache.give(b, f)) {
            if (f) f->wait();
            frees++;
            // the block leaves the cache's world: forget it (a real free)
            free(b.dev);
        }
    };
    std::atomic<int> next_pid{1};
    std::mutex handoff_mu;
    std::deque<std::pair<Blk, uint64_t>> handoff;
    std::atomic<bool> stop{false};
    std::thread cleaner([&] {   // a Handoff goroutine cleaning up others' processes
        for (;;) {
            std::pair<Blk, uint64_t> it;
            {
                std::lock_guard<std::mutex> lk(handoff_mu);
                if (handoff.empty()) {
                    if (stop) return;
                    it.first.dev = nullptr;
                } else {
                    it = handoff.front();
                    handoff.pop_front();
                }
            }
            if (!it.first.dev) {
                std::this_thread::yield();
                continue;
            }
            release(it.first, it.second);
        }
    });
    std::vector<std::thread> ts;
    for (int t = 0; t < 8; t++) {
        ts.emplace_back([&, t] {
            std::mt19937 rng(1234 + t);
            for (int k = 0; k < 400; k++) {
                const int pid = next_pid++;
                const size_t n = 1000 + rng() % 7000;
                Blk b;
                if (!cache.take(n, true, &b)) {
                    b.cls = BlkCache::size_class(n);
                    b.dev = (uint8_t *)malloc(b.cls);
                    b.host = b.dev;   // (a stand-in: the host half is not touched here)
                    allocs++;
                }
                BlockState *s = state_of(b.dev);
                int z = 0;
                CHECK(s->holder.compare_exchange_strong(z, pid), "block handed to process %d while process %d holds it", pid, z);
                CHECK(s->pending.load() == 0, "block handed out with %d work items of its last owner pending", s->pending.load());
                uint64_t last;
                {
                    std::lock_guard<std::recursive_mutex> lk(run_mu);
                    last = work_on(b.dev, pid);   // NewProcess's upload (no sync)
                }
                const unsigned what = rng() % 4;
                if (what != 0) {   // Run: a launch and the sync
                    std::lock_guard<std::recursive_mutex> lk(run_mu);
                    last = work_on(b.dev, pid);
                    sync();
                    CHECK(seq.idle(last), "a synced process is not idle");
                }
                if (what == 3) {   // cleaned up by the Handoff thread
                    std::lock_guard<std::mutex> lk(handoff_mu);
                    handoff.emplace_back(b, last);
                } else {
                    release(b, last);   // what == 0: the upload may still be queued
                }
            }
        });
    }
    for (auto &t : ts) t.join();
    stop = true;
    cleaner.join();
    st.wait_for(st.tail());
    CHECK(allocs > 0 && frees >= 0, "no allocations");
    cache.drain([](Blk &b) { free(b.dev); });
    printf("threads: %d allocations, %d freed past the cap\n", allocs.load(), frees.load());
}

int main() {
    test_fence_wait();
    test_cap();
    test_seqclock();
    test_threads();
    if (failures) {
        fprintf(stderr, "%d failures\n", failures.load());
        return 1;
    }
    printf("OK\n");
    return 0;
}

// blkcache.h -- host-side lifetime rules of single processes' memory (engine.cpp, NewProcess /
// Process.Cleanup, vm.go:198-235,363-374).  No HIP here: the engine plugs in its events, and
// tests/test_blkcache.py drives the same code with fake fences from many threads.
//
// Rules:
//  * A block given back carries the fence of its last use on the VM's stream, or none when that
//    use is known complete.  take() hands a block out only after its fence has passed, so a new
//    process never touches memory an older process's work may still read or write.
//  * Process operations that enqueue device work number their enqueues (SeqClock::next, under the
//    VM's run lock); a host sync of the stream completes every number up to the last one enqueued
//    before it (SeqClock::complete).  A process whose last number is complete needs no fence.
//  * Cleanup may run on any thread (processPool's Handoff goroutines, finalisers): the cache is
//    guarded by its own lock, never held across a wait.
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <atomic>
#include <map>
#include <memory>
#include <mutex>
#include <vector>

struct BlkFence {
    virtual ~BlkFence() {}
    virtual void wait() = 0;   // returns once the work the fence marks has completed
};

struct Blk {
    uint8_t *dev = nullptr;                    // device block
    uint8_t *host = nullptr, *hdev = nullptr;  // optional pinned host half and its device address
    size_t cls = 0;                            // size class (bytes of each half)
    std::shared_ptr<BlkFence> fence;           // last use still pending, or null
};

class BlkCache {
  public:
    explicit BlkCache(size_t cap_bytes) : cap_(cap_bytes) {}

    static size_t size_class(size_t n) {
        size_t c = 1024;
        while (c < n) c <<= 1;
        return c;
    }

    // a cached block of n bytes' class (with a host half when `host`), its fence waited for
    bool take(size_t n, bool host, Blk *out) {
        *out = Blk{};
        const size_t c = size_class(n);
        {
            std::lock_guard<std::mutex> lk(mu_);
            auto it = free_.find(key(c, host));
            if (it == free_.end() || it->second.empty()) return false;
            *out = std::move(it->second.back());
            it->second.pop_back();
            cached_ -= bytes(*out);
        }
        if (out->fence) out->fence->wait();   // outside the lock
        out->fence.reset();
        return true;
    }

    // give a block back with the fence of its last use; false: the cache is full and the caller
    // frees it (after waiting for the fence)
    bool give(const Blk &b, std::shared_ptr<BlkFence> fence) {
        if (!b.dev) return true;
        std::lock_guard<std::mutex> lk(mu_);
        if (cached_ + bytes(b) > cap_) return false;
        Blk c = b;
        c.fence = std::move(fence);
        free_[key(b.cls, b.host != nullptr)].push_back(std::move(c));
        cached_ += bytes(b);
        return true;
    }

    // every cached block, for freeing (the VM is being destroyed: its stream was synchronised)
    template <class F>
    void drain(F free_fn) {
        std::lock_guard<std::mutex> lk(mu_);
        for (auto &kv : free_)
            for (Blk &b : kv.second) free_fn(b);
        free_.clear();
        cached_ = 0;
    }

    size_t cached_bytes() {
        std::lock_guard<std::mutex> lk(mu_);
        return cached_;
    }

  private:
    static size_t key(size_t cls, bool host) { return cls | (host ? 1u : 0u); }
    static size_t bytes(const Blk &b) { return b.cls * (b.host ? 2 : 1); }
    std::mutex mu_;
    std::map<size_t, std::vector<Blk>> free_;
    size_t cached_ = 0;
    const size_t cap_;
};

// numbering of process enqueues on one stream (see the rules above)
struct SeqClock {
    std::atomic<uint64_t> enq{0}, done{0};
    uint64_t next() { return ++enq; }            // run lock held: a process enqueue was just made
    uint64_t issued() const { return enq.load(); }
    void complete(uint64_t upto) {                // a host sync covering every enqueue <= upto returned
        uint64_t d = done.load();
        while (d < upto && !done.compare_exchange_weak(d, upto)) {
        }
    }
    bool idle(uint64_t seq) const { return seq <= done.load(); }
};

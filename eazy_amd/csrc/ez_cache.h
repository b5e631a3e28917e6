// ez_cache.h — device scratch kept per (device, HIP stream) between batch calls.
//
// The batch entry points are asynchronous on the caller's HIP stream, so their scratch (K1's match
// records, K1c's logs, K2j's workspace) must outlive the call: it is kept per (device, stream) and
// grown as batches need.  Each entry has its own lock, held by a call from its first launch to its
// last: calls on distinct streams never wait for each other (the multi-device batches run a shard
// per host thread, and K1c's pass loop synchronises its own stream).  A stream the caller destroyed
// leaves its entry behind; entries beyond kMaxPerDevice on a device are freed least recently used
// first (hipFree waits for the device, so nothing still queued can use them), and trim() frees every
// idle entry of a device (ez_release_cached).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <atomic>
#include <map>
#include <memory>
#include <mutex>

namespace ez {

struct CacheEntry {
    std::mutex mu;          // held by the call using it
    std::atomic<int> refs{0};  // calls holding or waiting for mu (never evicted meanwhile)
    void *p = nullptr;
    size_t cap = 0;
    uint64_t used = 0;      // last use (the cache's tick)
    // grow-only, + 25 %; false when the allocation fails (the entry is then empty)
    bool ensure(size_t n) {
        if (n <= cap) return true;
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
        const size_t c = n < 4096 ? 4096 : n + n / 4;
        if (hipMalloc(&p, c) != hipSuccess) {
            (void)hipGetLastError();  // (not sticky: the caller may take a path without this scratch)
            return false;
        }
        cap = c;
        return true;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
    }
};

// a locked entry for the duration of one call
class CacheLease {
  public:
    CacheLease() = default;
    explicit CacheLease(CacheEntry *e) : e_(e) { e_->mu.lock(); }
    CacheLease(CacheLease &&o) noexcept : e_(o.e_) { o.e_ = nullptr; }
    CacheLease &operator=(CacheLease &&o) noexcept {
        done();
        e_ = o.e_;
        o.e_ = nullptr;
        return *this;
    }
    CacheLease(const CacheLease &) = delete;
    CacheLease &operator=(const CacheLease &) = delete;
    ~CacheLease() { done(); }
    CacheEntry *operator->() const { return e_; }
    CacheEntry *get() const { return e_; }

  private:
    void done() {
        if (!e_) return;
        e_->mu.unlock();
        e_->refs--;
        e_ = nullptr;
    }
    CacheEntry *e_ = nullptr;
};

class DevCache {
  public:
    static constexpr size_t kMaxPerDevice = 8;
    // the entry of (dev, stream), locked for the lease's lifetime (the caller's thread is bound to dev)
    CacheLease acquire(int dev, void *stream) {
        CacheEntry *e;
        {
            std::lock_guard<std::mutex> g(m_);
            auto &slot = map_[std::make_pair(dev, stream)];
            if (!slot) slot.reset(new CacheEntry());
            e = slot.get();
            e->used = ++tick_;
            e->refs++;
            evict_locked(dev);
        }
        return CacheLease(e);
    }
    // free every idle entry of dev (all devices for dev < 0) and drop it; the caller is bound to dev
    void trim(int dev) {
        std::lock_guard<std::mutex> g(m_);
        for (auto it = map_.begin(); it != map_.end();) {
            if ((dev < 0 || it->first.first == dev) && it->second->refs == 0 && it->second->mu.try_lock()) {
                it->second->release();
                it->second->mu.unlock();
                it = map_.erase(it);
            } else {
                ++it;
            }
        }
    }
    size_t entries(int dev) {
        std::lock_guard<std::mutex> g(m_);
        size_t k = 0;
        for (auto &kv : map_) k += kv.first.first == dev;
        return k;
    }

  private:
    // over kMaxPerDevice entries on dev: free the least recently used idle ones
    void evict_locked(int dev) {
        for (;;) {
            size_t n = 0;
            auto lru = map_.end();
            for (auto it = map_.begin(); it != map_.end(); ++it) {
                if (it->first.first != dev) continue;
                n++;
                if (it->second->refs == 0 && (lru == map_.end() || it->second->used < lru->second->used)) lru = it;
            }
            if (n <= kMaxPerDevice || lru == map_.end()) return;
            if (!lru->second->mu.try_lock()) return;  // (in use: kept until a later call)
            lru->second->release();
            lru->second->mu.unlock();
            map_.erase(lru);
        }
    }
    std::mutex m_;
    std::map<std::pair<int, void *>, std::unique_ptr<CacheEntry>> map_;
    uint64_t tick_ = 0;
};

}  // namespace ez

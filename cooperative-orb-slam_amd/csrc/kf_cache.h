/*
 * kf_cache.h -- the bookkeeping of orbm_kf_cache (include/orbslam_amd.h): an LRU map of keyframe entries over a
 * byte capacity, shared by every matcher thread of the process (the reference calls its matchers from Tracking,
 * LocalMapping and LoopClosing: Tracking.cc:767, LocalMapping.cc:268, LoopClosing.cc:267).
 *
 * Host-only and independent of HIP, so the same code runs in liborbamd.so (Entry = a keyframe's arrays in HBM) and
 * in the ThreadSanitizer test (tests/cpp/test_kf_cache_tsan.cpp, Entry = host memory). Entry provides
 * `size_t bytes() const`. Every member takes the one mutex; entries are handed out as shared_ptr, so a caller keeps
 * its entry alive (and its buffer allocated) after another thread evicts or replaces it, and the last reference
 * frees it. Two kinds of key space (0: matcher views, 1: projection views) share the LRU list and the capacity.
 */
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <list>
#include <memory>
#include <mutex>
#include <unordered_map>
#include <utility>

namespace orbamd {

template <class Entry>
class KfLru {
public:
    explicit KfLru(size_t capacity) : capacity_(capacity) {}

    /* the entry of (kind, key) if present and matches(entry) (moved to the front, counted a hit); a present entry
     * that does not match (the keyframe changed shape) is dropped; absent or dropped counts a miss -> nullptr */
    template <class Match>
    std::shared_ptr<Entry> find(int kind, uint64_t key, Match matches) {
        std::lock_guard<std::mutex> lock(mu_);
        auto& m = map_[kind];
        auto it = m.find(key);
        if (it != m.end()) {
            if (matches(*it->second.e)) {
                hits_++;
                lru_.splice(lru_.begin(), lru_, it->second.lru);
                return it->second.e;
            }
            drop(m, it);  // in-flight calls keep their shared_ptr; the buffer goes with the last one
        }
        misses_++;
        return nullptr;
    }

    /* inserts e (built by the caller outside the lock after a miss) and returns the entry to use: an entry another
     * thread inserted meanwhile wins if it matches (both uploaded; the first one is shared), else it is replaced.
     * Then evicts least recently used entries while over capacity, never the one returned. */
    template <class Match>
    std::shared_ptr<Entry> insert(int kind, uint64_t key, std::shared_ptr<Entry> e, Match matches) {
        std::lock_guard<std::mutex> lock(mu_);
        auto& m = map_[kind];
        auto it = m.find(key);
        if (it != m.end()) {
            if (matches(*it->second.e)) {
                lru_.splice(lru_.begin(), lru_, it->second.lru);
                return it->second.e;
            }
            drop(m, it);
        }
        lru_.push_front({kind, key});
        m[key] = Slot{e, lru_.begin()};
        bytes_ += e->bytes();
        while (bytes_ > capacity_ && lru_.size() > 1) {
            const auto victim = lru_.back();
            auto& vm = map_[victim.first];
            drop(vm, vm.find(victim.second));
        }
        return e;
    }

    /* KeyFrame::SetBadFlag (amd::ForgetKeyFrame): drop the key in both key spaces */
    void erase(uint64_t key) {
        std::lock_guard<std::mutex> lock(mu_);
        for (auto& m : map_) {
            auto it = m.find(key);
            if (it != m.end()) drop(m, it);
        }
    }

    void stats(int* entries, size_t* bytes, long long* hits, long long* misses) {
        std::lock_guard<std::mutex> lock(mu_);
        if (entries) *entries = (int)(map_[0].size() + map_[1].size());
        if (bytes) *bytes = bytes_;
        if (hits) *hits = hits_;
        if (misses) *misses = misses_;
    }

    /* consistency of the books (tests): the byte count equals the entries' sizes, the LRU list holds exactly the
     * mapped keys, and the capacity holds unless a single entry exceeds it */
    bool consistent() {
        std::lock_guard<std::mutex> lock(mu_);
        size_t b = 0, n = 0;
        for (auto& m : map_)
            for (auto& kv : m) {
                b += kv.second.e->bytes();
                n++;
            }
        return b == bytes_ && n == lru_.size() && (bytes_ <= capacity_ || lru_.size() <= 1);
    }

    void clear() {
        std::lock_guard<std::mutex> lock(mu_);
        map_[0].clear();
        map_[1].clear();
        lru_.clear();
        bytes_ = 0;
    }

private:
    struct Slot {
        std::shared_ptr<Entry> e;
        std::list<std::pair<int, uint64_t>>::iterator lru;
    };
    using Map = std::unordered_map<uint64_t, Slot>;
    void drop(Map& m, typename Map::iterator it) {
        bytes_ -= it->second.e->bytes();
        lru_.erase(it->second.lru);
        m.erase(it);
    }

    std::mutex mu_;
    size_t capacity_;
    Map map_[2];
    std::list<std::pair<int, uint64_t>> lru_;  // front = most recently used
    size_t bytes_ = 0;
    long long hits_ = 0, misses_ = 0;
};

}  // namespace orbamd
